"""Pins the CPU oracle (oracle/gnpde_oracle.py) against the reference.

* every golden fixture in tests/golden/ (made by tests/golden/gen_golden.py from
  the reference's own modules, float64);
* the reference tests' known answers: test/test_utils.py:62-79 (rw adjacency
  == sklearn.normalize(A + s I)), test/test_function_laplacian_diffusion.py:56-86
  (rw and symmetric adjacency on the toy graph),
  test/test_transformer_attention.py:44-106 (attention sums to 1 per group,
  0 < att <= 1, complete 3-graph with x = ones -> 0.5) and :118-143 (head-mean
  equivalence);
* the O(E*d) global-key-sum restatement of the fork's scaled_dot
  equals the literal [h,E,E] matmul formula.
"""
import glob
import json
import os

import numpy as np
import pytest

import gnpde_oracle as O
from conftest import GOLDEN

FIXTURES = sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load(path):
    d = np.load(path, allow_pickle=False)
    return d, json.loads(str(d["meta"]))


def rel(a, b):
    den = max(np.abs(b).max(), 1e-30)
    return np.abs(np.asarray(a, np.float64) - b).max() / den


def oracle_rhs(d, m):
    if m["kind"] == "laplacian":
        kw = dict(edge_weight=d["weights"]) if m["block"] == "constant" else dict(attention_weights=d["weights"])
        return O.laplacian_rhs(d["edge_index"], d["x"], d["x0"], d["alpha_train"], d["beta_train"], block=m["block"],
                               add_source=m["add_source"], no_alpha_sigmoid=m["no_alpha_sigmoid"], **kw)
    return O.transformer_rhs(d["edge_index"], d["x"], d["x0"], d["Wq"], d["bq"], d["Wk"], d["bk"], m["heads"],
                             m["attention_norm_idx"], d["alpha_train"], d["beta_train"],
                             attention_type=m["attention_type"], add_source=m["add_source"],
                             no_alpha_sigmoid=m["no_alpha_sigmoid"], output_var=m["output_var"] or 1.0,
                             lengthscale=m["lengthscale"] or 1.0)


def test_fixture_manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as fh:
        names = json.load(fh)
    assert sorted(os.path.basename(p)[:-4] for p in FIXTURES) == sorted(names)
    assert len(names) >= 20


@pytest.mark.parametrize("path", [p for p in FIXTURES if os.path.basename(p).startswith(("lap_", "att_"))],
                         ids=os.path.basename)
def test_oracle_rhs_matches_reference(path):
    d, m = load(path)
    f = oracle_rhs(d, m)
    assert f.shape == d["f"].shape
    # fp64 restatement vs the fp64 reference: only summation order differs
    assert rel(f, d["f"]) < 1e-12


@pytest.mark.parametrize("path", [p for p in FIXTURES if os.path.basename(p).startswith("att_")],
                         ids=os.path.basename)
def test_oracle_attention_matches_reference(path):
    d, m = load(path)
    att = O.transformer_attention(d["x"], d["edge_index"], d["Wq"], d["bq"], d["Wk"], d["bk"], m["heads"],
                                  m["attention_norm_idx"], attention_type=m["attention_type"],
                                  output_var=m["output_var"] or 1.0, lengthscale=m["lengthscale"] or 1.0)
    assert np.abs(att - d["attention"]).max() < 1e-12
    prods = O.attention_scores(d["x"], d["edge_index"], d["Wq"], d["bq"], d["Wk"], d["bk"], m["heads"],
                               m["attention_type"], output_var=m["output_var"] or 1.0,
                               lengthscale=m["lengthscale"] or 1.0)
    assert rel(prods, d["prods"]) < 1e-12


@pytest.mark.parametrize("path", [p for p in FIXTURES if "softmax" in p], ids=os.path.basename)
def test_oracle_softmax_matches_reference(path):
    d, _ = load(path)
    assert np.abs(O.edge_softmax(d["src"], d["index"]) - d["out"]).max() < 1e-15


@pytest.mark.parametrize("path", [p for p in FIXTURES if os.path.basename(p).startswith("mixed_")],
                         ids=os.path.basename)
def test_oracle_mixed_attention_matches_reference(path):
    """MixedODEblock.get_mixed_attention (src/block_mixed.py:29-33), reference fp64 run."""
    d, _ = load(path)
    w = O.mixed_attention(d["attention"], d["edge_weight"], d["gamma"])
    assert np.abs(w - d["w"]).max() < 1e-14
    assert np.abs(d["w_ref32"] - d["w"]).max() < 1e-6


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 4097])
@pytest.mark.parametrize("q", [0.0, 0.1, 0.25, 0.5, 0.9, 1.0])
def test_oracle_quantile_matches_torch(n, q):
    """torch.quantile (the threshold of src/block_transformer_hard_attention.py:52), in-container torch."""
    torch = pytest.importorskip("torch")
    v = np.random.default_rng(n).standard_normal(n).astype(np.float32)
    want = float(torch.quantile(torch.from_numpy(v), q))
    assert float(O.quantile_f32(v, q)) == want


@pytest.mark.parametrize("norm_idx", [0, 1])
def test_oracle_hard_attention_sample(norm_idx):
    """Kept edges exceed the quantile threshold, each group of the kept graph sums to 1."""
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(3 + norm_idx)
    N, E = 50, 600
    ei = rng.integers(0, N, size=(1, 2, E))
    att = rng.uniform(0, 1, (1, E, 2)).astype(np.float32)
    ei2, w = O.hard_attention_sample(ei, att, 0.4, norm_idx, N)
    mean = att.mean(axis=2)
    thr = float(torch.quantile(torch.from_numpy(mean), 0.6))
    assert ei2.shape[2] == int((mean[0] > thr).sum()) and 0 < ei2.shape[2] < E
    sums = np.zeros(N)
    np.add.at(sums, ei2[0, norm_idx], w[0])
    live = np.unique(ei2[0, norm_idx])
    assert np.allclose(sums[live], 1.0, atol=1e-12)


def test_reference_fp32_within_tolerance_of_fp64():
    """The reference's own fp32 run sits within the 1e-5 parity tolerance of its fp64 run."""
    worst = 0.0
    for p in FIXTURES:
        d, m = load(p)
        if "f_ref32" in d and np.abs(d["f"]).max() > 0:
            worst = max(worst, rel(d["f_ref32"], d["f"]))
    assert worst < 1e-5


# ---------------------------------------------------------------- known answers
EDGE_UTILS = np.array([[[0, 2, 2, 1], [1, 0, 1, 2]]])       # test/test_utils.py:37
EDGE_LAP = np.array([[[0, 1, 2, 1], [1, 0, 1, 2]]])         # test/test_function_laplacian_diffusion.py:33


def _dense(eis, ws, n):
    return O.to_dense(eis[0], ws[0], n)


@pytest.mark.parametrize("self_loop", [0, 0.3, 1, 3.2])
@pytest.mark.parametrize("norm_dim", [0, 1])
def test_kat_rw_adj(self_loop, norm_dim):
    """test/test_utils.py:62-79."""
    from sklearn.preprocessing import normalize
    base = O.to_dense(EDGE_UTILS[0], np.ones(4), 3)
    want = normalize(base + np.identity(3) * self_loop, norm="l1", axis=0 if norm_dim == 1 else 1)
    eis, ws = O.get_rw_adj(EDGE_UTILS, norm_dim=norm_dim, fill_value=self_loop, num_nodes=3)
    assert np.allclose(_dense(eis, ws, 3), want)


def test_kat_laplacian_block_toy():
    """test/test_function_laplacian_diffusion.py:56-86 (rw and symmetric adjacency)."""
    from sklearn.preprocessing import normalize
    aug = O.to_dense(EDGE_LAP[0], np.ones(4), 3) + np.identity(3)
    eis, ws = O.get_rw_adj(EDGE_LAP, norm_dim=1, fill_value=1, num_nodes=3)
    assert np.allclose(_dense(eis, ws, 3), normalize(aug, norm="l1", axis=0))
    deg = np.sqrt(aug.sum(axis=1))
    eis, ws = O.gcn_norm_fill_val(EDGE_LAP, fill_value=1, num_nodes=3)
    assert np.allclose(_dense(eis, ws, 3), aug / deg[:, None] / deg[None, :])


def test_kat_symmetric_attention_half():
    """test/test_transformer_attention.py:98-106: x = ones, complete 3-graph -> 0.5."""
    d, m = load(os.path.join(GOLDEN, "att_kat_symmetric.npz"))
    att = O.transformer_attention(d["x"], d["edge_index"], d["Wq"], d["bq"], d["Wk"], d["bk"], 2, 0)
    assert np.all(att == 0.5)


@pytest.mark.parametrize("norm_idx", [0, 1])
def test_property_attention_group_sums(norm_idx):
    """test/test_transformer_attention.py:57-76: per-group sums round to 1, 0 < att <= 1."""
    rng = np.random.default_rng(3)
    N, E, C, h, att = 30, 200, 6, 2, 8
    ei = rng.integers(0, N, size=(1, 2, E))
    x = rng.standard_normal((1, N, C))
    W = [rng.standard_normal((att, C)) * 0.2, rng.standard_normal(att) * 0.2] * 2
    a = O.transformer_attention(x, ei, W[0], W[1], W[2], W[3], h, norm_idx, score_mode="per_edge")
    for hh in range(h):
        sums = np.zeros(N)
        np.add.at(sums, ei[0, norm_idx], a[0, :, hh])
        live = np.unique(ei[0, norm_idx])
        assert np.allclose(np.round(sums[live], 3), 1.0)
    assert np.all(a > 0) and np.all(a <= 1)


def test_head_mean_equivalence():
    """test/test_transformer_attention.py:118-143: mean over heads of per-head
    aggregations == aggregation with the mean attention."""
    rng = np.random.default_rng(5)
    N, E, C, h = 20, 90, 4, 3
    ei = rng.integers(0, N, size=(1, 2, E))
    x = rng.standard_normal((1, N, C))
    att = rng.uniform(size=(1, E, h))
    per_head = np.mean([O.aggregate(ei, att[:, :, k], x) for k in range(h)], axis=0)
    assert np.allclose(per_head, O.aggregate(ei, att.mean(axis=2), x))


def test_fork_scaled_dot_global_key_sum():
    """sum(matmul(src[B,h,E,dk], dst_k[B,h,dk,E]/sqrt(dk)), 3) (the literal
    function_transformer_attention.py:249) == q_src . sum_e' k_dst(e') / sqrt(dk)."""
    rng = np.random.default_rng(7)
    N, E, C, h, att = 15, 40, 5, 2, 8
    ei = rng.integers(0, N, size=(2, 2, E))
    x = rng.standard_normal((2, N, C))
    Wq, bq, Wk, bk = (rng.standard_normal((att, C)), rng.standard_normal(att), rng.standard_normal((att, C)),
                      rng.standard_normal(att))
    q = O.split_heads(O.project(x, Wq, bq), h)
    k = O.split_heads(O.project(x, Wk, bk), h)
    dk = att // h
    lit = np.zeros((2, E, h))
    for b in range(2):
        src = q[b][ei[b, 0]].transpose(2, 0, 1)         # [h,E,dk]
        dst = k[b][ei[b, 1]].transpose(2, 1, 0) / np.sqrt(dk)  # [h,dk,E]
        lit[b] = np.matmul(src, dst).sum(axis=2).T
    got = O.attention_scores(x, ei, Wq, bq, Wk, bk, h, "scaled_dot", "reference")
    assert rel(got, lit) < 1e-12
    # with norm_idx = 0 every edge of a source row gets 1/outdeg
    a = O.edge_softmax(got, ei[:, 0])
    outdeg = np.zeros((2, N))
    for b in range(2):
        np.add.at(outdeg[b], ei[b, 0], 1)
        assert np.allclose(a[b, :, 0], 1.0 / outdeg[b][ei[b, 0]])


def test_oracle_fixed_grid_matches_torchdiffeq_formula():
    g = O.fixed_grid(0.0, 1.0, 0.1)
    assert len(g) == 11 and g[0] == 0 and g[-1] == np.float32(1.0)
    assert len(O.fixed_grid(0.0, 1.0, 1.0)) == 2
    assert len(O.fixed_grid(0.0, 3.0, 0.25)) == 13


def test_oracle_rk4_on_linear_ode():
    """rk4 (3/8 rule) on y' = -y: global error O(h^4)."""
    f = lambda t, y: -y  # noqa: E731
    y = O.odeint_fixed(f, np.ones(3), 0.0, 1.0, "rk4", 0.1)
    assert np.allclose(y, np.exp(-1.0), atol=1e-6)
    y = O.odeint_fixed(f, np.ones(3), 0.0, 1.0, "euler", 0.1)
    assert np.allclose(y, 0.9 ** 10)


# ---------------------------------------------------------------- reference gradient fixtures
GRADS = sorted(glob.glob(os.path.join(GOLDEN, "grad_*.npz")))


@pytest.mark.parametrize("path", GRADS, ids=os.path.basename)
def test_grad_fixture_is_the_oracle_derivative(path):
    """The reference-autograd gradient fixtures agree with central differences
    of the ORACLE's forward (fp64) along random directions: pins them to the
    same function the oracle restates, independently of torch autograd."""
    d = np.load(path, allow_pickle=False)
    m = json.loads(str(d["meta"]))
    rng = np.random.default_rng(3)
    gout = d["gout"].astype(np.float64)
    base = {k: d[k].astype(np.float64) for k in ("x", "alpha_train", "beta_train")}
    if m["kind"] == "laplacian_grad":
        base["weights"] = d["weights"].astype(np.float64)

        def loss(v):
            f = O.laplacian_rhs(d["edge_index"], v["x"], d["x0"], float(v["alpha_train"]), float(v["beta_train"]),
                                block=m["block"], edge_weight=v["weights"], attention_weights=v["weights"],
                                add_source=m["add_source"], no_alpha_sigmoid=m["no_alpha_sigmoid"])
            return float((f * gout).sum())
    else:
        for k in ("Wq", "bq", "Wk", "bk"):
            base[k] = d[k].astype(np.float64)
        kw = {}
        if m["attention_type"] == "exp_kernel":
            base["output_var"] = np.float64(m["output_var"])
            base["lengthscale"] = np.float64(m["lengthscale"])

        def loss(v):
            if m["attention_type"] == "exp_kernel":
                kw.update(output_var=float(v["output_var"]), lengthscale=float(v["lengthscale"]))
            f = O.transformer_rhs(d["edge_index"], v["x"], d["x0"], v["Wq"], v["bq"], v["Wk"], v["bk"], m["heads"],
                                  m["attention_norm_idx"], float(v["alpha_train"]), float(v["beta_train"]),
                                  attention_type=m["attention_type"], add_source=m["add_source"],
                                  no_alpha_sigmoid=m["no_alpha_sigmoid"], **kw)
            return float((f * gout).sum())
    for name in base:
        key = "g_" + name
        if key not in d.files:
            continue
        g = d[key].astype(np.float64)
        u = rng.standard_normal(np.shape(base[name]))
        eps = 1e-5 * max(1.0, float(np.abs(base[name]).max()))
        vp = dict(base)
        vm = dict(base)
        vp[name] = base[name] + eps * u
        vm[name] = base[name] - eps * u
        fd = (loss(vp) - loss(vm)) / (2 * eps)
        an = float((g * u).sum())
        assert abs(fd - an) <= 1e-6 * max(1.0, abs(an)) + 1e-7 * float(np.abs(g).sum()), (name, fd, an)
