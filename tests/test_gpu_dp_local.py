"""The engine's data-parallel decomposition on ONE GPU, without RCCL (-m gpu).

mmvae_comm_init(h, rank, world, NULL) puts a handle in the local decomposition mode: it runs
rank r's shard of a world-W step exactly as under RCCL — loss and gradients divided by the
GLOBAL batch (n_total), reparameterisation noise keyed by the global row (row_offset + batch
position), the vMF lbessel backward (Q3, independent of the upstream gradient) added on rank 0
only — but reduces nothing.  Summing the shards' losses and gradients on the host must give the
single-engine step over the whole batch: this checks the kernels' share of the
DP path; the RCCL bucket exchange itself needs two GPUs (unmeasured on this pool).
"""
import numpy as np
import pytest

from helpers import rel_err

pytestmark = pytest.mark.gpu


def _engine(model, D, K, B, dtype, relu=False):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=9, relu=relu, model=MODEL_VMF if model == "vmf" else MODEL_NB)
    eng.synth_csr(3000, lib_size=1500.0, seed=4)
    eng.init_params(seed=13)
    if model == "vmf":
        eng.set_param("ln_kappa", np.array([np.log(np.float32(3.0))], np.float32))
    return eng


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_local_dp_shards_sum_to_single_step(model, world):
    D, K, B = 3000, 32, 512
    cells = (np.arange(B, dtype=np.int64) * 5 + 3) % 3000
    full = _engine(model, D, K, B, "f32")
    l_full, n_full = full.step(cells, 0.7, step_id=5)
    g_full = full.grads()
    b = B // world
    losses, gsum = [], None
    for r in range(world):
        eng = _engine(model, D, K, b, "f32")
        eng.comm_init(r, world, None)
        l, _ = eng.step(cells[r * b:(r + 1) * b], 0.7, n_total=B, row_offset=r * b, step_id=5)
        losses.append(l)
        g = eng.grads()
        gsum = g if gsum is None else {k: gsum[k] + g[k] for k in g}
    assert abs(sum(losses) - l_full) <= 2e-5 * abs(l_full), (sum(losses), l_full)
    for k in g_full:
        if k == "ln_kappa":  # fp32 cancellation of df/kappa-sized terms (see test_gpu_vmf.py)
            assert abs(float(gsum[k][0] - g_full[k][0])) <= 1e-6 * (0.5 * D - 1.0), (gsum[k], g_full[k])
            continue
        assert rel_err(gsum[k], g_full[k]) <= 2e-5, (k, rel_err(gsum[k], g_full[k]))
    # clip_grad_norm_ of the all-reduced gradient = the single step's total norm
    tot = np.sqrt(sum(float(np.sum(np.asarray(v, np.float64) ** 2)) for v in gsum.values()))
    assert abs(tot - n_full) <= 2e-5 * n_full, (tot, n_full)


def test_vmf_baricz_term_on_rank0_only():
    """Q3: the lbessel backward ignores its upstream gradient, so a shard's ln_kappa gradient
    differs between rank 0 and the others by exactly Baricz(kappa) * kappa."""
    from mmvae_amd import lbessel_grad
    D, K, B = 3000, 32, 256
    cells = np.arange(B, dtype=np.int64)
    out = {}
    for r in (0, 1):
        eng = _engine("vmf", D, K, B, "f32")
        eng.comm_init(r, 2, None)
        eng.step(cells, 0.7, n_total=2 * B, row_offset=0, step_id=1)
        out[r] = float(eng.get_grad("ln_kappa", 1)[0])
    kap = np.float32(3.0)
    want = lbessel_grad(float(kap), 0.5 * D - 1.0) * float(kap)
    assert abs((out[0] - out[1]) - want) <= 1e-4 * abs(want), (out, want)


@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_local_dp_step_graphs_replay_and_match_eager(model):
    """A17 under DP: shards of a world-2 step run as replayed step graphs (mmvae_graph_stats)
    and give bit-identical losses and gradients to the same shards launched eagerly."""
    D, K, B, world = 3000, 32, 512, 2
    b = B // world
    out = {}
    for graph in (False, True):
        res = []
        for r in range(world):
            eng = _engine(model, D, K, b, "bf16x3")
            eng.comm_init(r, world, None)
            eng.graph(graph)
            for s in range(4):
                cells = (np.arange(B, dtype=np.int64) * 7 + 11 * s) % 3000
                l, n = eng.step(cells[r * b:(r + 1) * b], 0.7, n_total=B, row_offset=r * b, step_id=s)
                res.append((l, n))
            res.append(eng.grads())
            if graph:
                st = eng.graph_stats()
                assert st["replays"] == 4 and st["captures"] >= 1, st
            eng.close()
        out[graph] = res
    for a, c in zip(out[False], out[True]):
        if isinstance(a, dict):
            for k in a:
                assert np.array_equal(a[k], c[k]), k
        else:
            assert a == c, (a, c)
