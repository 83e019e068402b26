"""MultiFusion scoring surface (combiner.py / validate.py / inference.py) on libcmve.so."""
