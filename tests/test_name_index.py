"""Host logic of MultiFusion's ranking (no GPU): cirr_target_ranks turns index / reference / target names into
gallery rows as the reference's name lookups do (MultiFusion/src/validate.py:71-105 -- `index_names.index(...)`
style lookups over a name list): the row of a name, the LAST row of a repeated name (a {name: row} dict built in
order), -1 for a name that is not in the gallery.  Both of _NameIndex's forms are checked against that dict: the
direct table (dense non-negative integer ids) and the sorted search (sparse or negative ids, numeric strings)."""
import numpy as np
import pytest

from cmve.multifusion import validate as V


def _dict_rows(index_names, names):
    d = {}
    for i, v in enumerate(index_names):
        d[int(v)] = i
    return [d.get(int(x), -1) for x in names]


@pytest.mark.parametrize("case", ["dense", "dense_repeats", "sparse", "negative", "strings", "numpy", "empty"])
def test_name_index_matches_dict(case):
    rng = np.random.default_rng(7)
    if case == "dense":
        idx = list(rng.permutation(5000))
    elif case == "dense_repeats":
        idx = list(rng.integers(0, 3000, 5000))
    elif case == "sparse":
        idx = list(rng.choice(10 ** 12, 3000, replace=False))
    elif case == "negative":
        idx = list(rng.integers(-50, 2000, 3000))
    elif case == "strings":
        idx = [str(x) for x in rng.integers(0, 4000, 3000)]
    elif case == "numpy":
        idx = rng.integers(0, 4000, 3000)
    else:
        idx = []
    pool = [int(x) for x in idx] + [-7, 10 ** 12 + 5, 4_000_000]
    names = [pool[k] for k in rng.integers(0, len(pool), 2000)] if pool else [1, 2, 3]
    if case == "strings":
        names = [str(x) for x in names]
    ix = V._NameIndex(idx)
    assert (ix.lut is not None) == (case in ("dense", "dense_repeats", "strings", "numpy"))
    got = ix.rows(names)
    assert list(got) == _dict_rows(idx, names)
