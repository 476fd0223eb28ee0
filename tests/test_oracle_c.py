"""The C restatement (oracle/c/rhs_oracle.c, the timed CPU baseline) agrees with
the numpy oracle, which tests/test_oracle_golden.py pins to the reference."""
import glob
import json
import os
import subprocess

import numpy as np
import pytest

import gnpde_oracle as O
from conftest import GOLDEN, ROOT


@pytest.fixture(scope="module")
def coracle():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    return O.COracle()


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "lap_*.npz"))), ids=os.path.basename)
def test_c_oracle_matches_golden(coracle, path):
    d = np.load(path, allow_pickle=False)
    m = json.loads(str(d["meta"]))
    w = O.laplacian_weights(m["block"], d["weights"], d["weights"]).astype(np.float32)
    csr = coracle.csr(d["edge_index"], w, m["N"])
    f = coracle.laplacian_rhs(csr, d["x"], float(d["alpha_train"]), d["x0"], float(d["beta_train"]),
                              m["no_alpha_sigmoid"], m["add_source"], nthreads=2)
    assert np.abs(f - d["f"]).max() / np.abs(d["f"]).max() < 1e-5


def test_c_oracle_csr_is_stable_and_validates(coracle):
    ei = np.array([[[2, 0, 2, 1], [0, 1, 1, 2]]])
    rowptr, col, w = coracle.csr(ei, np.array([[1.0, 2.0, 3.0, 4.0]]), 3)
    assert rowptr.tolist() == [0, 1, 2, 4] and col.tolist() == [1, 2, 0, 1] and w.tolist() == [2.0, 4.0, 1.0, 3.0]
    with pytest.raises(ValueError):
        coracle.csr(np.array([[[0], [5]]]), np.ones((1, 1)), 3)
