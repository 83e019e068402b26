"""LINAS-engine retrieval surface (evaluation.py / util/metrics.py / validate.py / inference.py)."""
