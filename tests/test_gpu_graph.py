"""Step graphs (one hipGraph per step, -m gpu).

With mmvae_graph_enable the handle captures a step's device work (the staged H2D copy, every
kernel, the loss readback) once per launch shape and replays it; the per-step scalars (Philox
step / global row offset, Adam's bias corrections) travel in the staged copy.  A graph handle and
an eager handle driven through the same sequence — shape changes (ragged last batch, n_total,
beta, eval, injected eps) included — must agree BIT FOR BIT in losses, norms and parameters, and the graph handle must have replayed instead of re-captured.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _engine(model, D, K, B, dtype, graph, **kw):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=9, model=MODEL_VMF if model == "vmf" else MODEL_NB, **kw)
    eng.synth_csr(3000, lib_size=1500.0, seed=4)
    eng.init_params(seed=13)
    eng.graph(graph)
    return eng


@pytest.mark.parametrize("model,dtype", [("nb", "f32"), ("nb", "bf16x3"), ("nb", "bf16"), ("vmf", "bf16x3")])
def test_graph_steps_bit_identical_to_eager(model, dtype):
    D, K, B = 3000, 32, 256
    rng = np.random.default_rng(0)
    seq = []  # (kind, cells, beta, n_total, row_offset, eps)
    for i in range(4):
        seq.append(("step", rng.integers(0, 3000, B), 1.0, B, 0, None))
    seq.append(("step", rng.integers(0, 3000, 100), 1.0, 100, 0, None))     # ragged batch: new shape
    seq.append(("step", rng.integers(0, 3000, B), 0.5, B, 0, None))         # beta change: new shape
    seq.append(("eval", rng.integers(0, 3000, B), 0.5, B, 0, None))
    seq.append(("step", rng.integers(0, 3000, B), 0.5, 4 * B, 3 * B, None))  # DP-style shard scalars
    eps = rng.standard_normal(B * (K + (0 if model == "vmf" else 1))).astype(np.float32)
    seq.append(("step", rng.integers(0, 3000, B), 0.5, B, 0, eps))
    for i in range(3):
        seq.append(("step", rng.integers(0, 3000, B), 1.0, B, 0, None))    # back to the first shape
    out = []
    for graph in (False, True):
        eng = _engine(model, D, K, B, dtype, graph)
        trace = []
        for i, (kind, cells, beta, n_total, ro, ep) in enumerate(seq):
            if kind == "eval":
                trace.append((eng.eval_loss(cells, beta, step_id=100 + i), 0.0))
            else:
                trace.append(eng.step(cells, beta, n_total=n_total, row_offset=ro, step_id=100 + i, eps=ep))
        out.append((trace, eng.params(), eng.graph_stats()))
    (t0, p0, s0), (t1, p1, s1) = out
    assert s0 == {"captures": 0, "replays": 0}
    assert s1["replays"] == len(seq)
    # shapes: base, ragged, beta, eval, shard, eps, base again; one graph per pinned staging slot
    assert s1["captures"] <= 12, s1
    assert t0 == t1                          # losses and norms, bit for bit
    for k in p0:
        assert np.array_equal(p0[k], p1[k]), k


def test_graph_bench_shape_identical_and_timed():
    """The bench's NB step (D = 20000, B = 4096, latent 64) with and without graphs: identical
    results; the per-step times are printed for the record (launch gaps are a few us)."""
    import time
    D, K, B = 20000, 64, 4096
    res = []
    for graph in (False, True):
        from mmvae_amd import Engine
        eng = Engine(D=D, K=K, max_batch=B, dtype="bf16", seed=1)
        eng.synth_csr(20000, lib_size=2000.0, seed=3)
        eng.init_params(seed=7)
        eng.graph(graph)
        cells = [np.random.default_rng(s).integers(0, 20000, B) for s in range(12)]
        losses = [eng.step(cells[i], 1.0, step_id=i) for i in range(4)]
        eng.sync()
        t = time.perf_counter()
        for i in range(4, 12):
            eng.step(cells[i], 1.0, step_id=i, sync=False)
        eng.sync()
        dt = (time.perf_counter() - t) / 8
        res.append((losses, eng.params(), dt))
        if graph:
            assert eng.graph_stats() == {"captures": 2, "replays": 12}  # one per staging slot
        print(f"graph={graph}: {dt * 1e3:.3f} ms/step")
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


@pytest.mark.parametrize("model,dtype", [("nb", "f32"), ("nb", "bf16x3"), ("vmf", "bf16x3")])
def test_ragged_batch_independent_of_handle_capacity(model, dtype):
    """A ragged batch (B = 100: padded to 128 rows) on a handle sized for 512 rows: the latent
    kernels run over every row of the handle, and rows past this batch's padded size must not
    touch the batch's [KP][Bpad] operand images (dh^T, and z's x3 lo plane) — they once raced
    with the real rows.  Repeated 512-row handles agree bit for bit; a 128-row handle (other gene
    splits, so other fixed summation orders) agrees to rounding."""
    from helpers import rel_err
    D, K = 3000, 32
    cells = (np.arange(100, dtype=np.int64) * 29 + 5) % 3000
    runs = []
    for cap in (512, 512, 512, 128):
        eng = _engine(model, D, K, cap, dtype, False)
        out = eng.step(cells, 1.0, step_id=3)
        runs.append((out, eng.grads()))
    for out, g in runs[1:3]:
        assert out == runs[0][0]
        for k in g:
            assert np.array_equal(g[k], runs[0][1][k]), (k, float(np.abs(g[k] - runs[0][1][k]).max()))
    out, g = runs[3]
    assert abs(out[0] - runs[0][0][0]) <= 1e-6 * abs(out[0])
    for k in g:
        assert rel_err(g[k], runs[0][1][k]) <= 1e-5, (k, rel_err(g[k], runs[0][1][k]))


def _sequence(model, K, B, seed=0):
    rng = np.random.default_rng(seed)
    seq = [("step", rng.integers(0, 3000, B), 1.0, B, 0, None) for _ in range(2)]
    seq.append(("step", rng.integers(0, 3000, 100), 1.0, 100, 0, None))      # ragged (padded rows)
    seq.append(("eval", rng.integers(0, 3000, B), 0.5, B, 0, None))
    seq.append(("step", rng.integers(0, 3000, 37), 0.5, 4 * B, 3 * B, None))  # ragged DP shard
    eps = rng.standard_normal(B * (K + (0 if model == "vmf" else 1))).astype(np.float32)
    seq.append(("step", rng.integers(0, 3000, B), 0.5, B, 0, eps))
    seq.append(("step", rng.integers(0, 3000, B), 1.0, B, 0, None))
    return seq


HIDDEN = {"enc_hidden": (48,), "dec_hidden": (40, 24)}


@pytest.mark.parametrize("model,dtype,arch", [("nb", "f32", {}), ("nb", "bf16x3", {}), ("nb", "bf16", {}),
                                              ("nb", "fp8", {}), ("vmf", "f32", {}), ("vmf", "bf16x3", {}),
                                              ("vmf", "bf16", {}), ("nb", "bf16x3", HIDDEN),
                                              ("vmf", "bf16x3", dict(HIDDEN, relu=True))],
                         ids=lambda v: "hidden" if isinstance(v, dict) and v else ("" if isinstance(v, dict) else v))
def test_poisoned_workspace_bit_identical(model, dtype, arch):
    """Every per-step workspace buffer (batch lists, tile offsets, split partials, latent
    records, operand images, column slabs, loss / norm partials) is overwritten between steps
    with NaN bytes (0xFF) or huge finite floats (0x7F) — mmvae_debug_poison.  A step that reads
    a word it did not write this step (a stale padding row, an unwritten split partial) then
    changes the result; every loss, norm and parameter must stay bit-identical to the unpoisoned
    run, eager and graph alike.  This is the check behind the round-2 ragged-batch mismatch."""
    D, K, B = 3000, 32, 256
    seq = _sequence(model, K, B)
    out = []
    for poison, graph in ((None, False), (0xFF, False), (0x7F, True)):
        eng = _engine(model, D, K, B, dtype, graph, **arch)
        trace = []
        for i, (kind, cells, beta, n_total, ro, ep) in enumerate(seq):
            if poison is not None:
                eng.poison(poison)
            if kind == "eval":
                trace.append((eng.eval_loss(cells, beta, step_id=100 + i), 0.0))
            else:
                trace.append(eng.step(cells, beta, n_total=n_total, row_offset=ro, step_id=100 + i, eps=ep))
        out.append((trace, eng.params()))
    for trace, params in out[1:]:
        assert trace == out[0][0]
        for k in params:
            assert np.array_equal(params[k], out[0][1][k]), k


@pytest.mark.parametrize("model,dtype", [("nb", "f32"), ("nb", "bf16x3"), ("nb", "bf16"), ("vmf", "bf16x3")])
def test_repeated_ragged_step_deterministic(model, dtype):
    """Race detector: the same ragged step (B = 100 on a 256-row handle) run eight times on one
    handle from the same parameters and optimiser state, the workspace poisoned differently
    before each run.  Every cross-wave / cross-workgroup sum is a fixed-order reduction of plain
    stores, so loss, clip norm and every gradient must repeat bit for bit; an LDS or global race
    (a read racing a write of another wave) shows up as run-to-run drift."""
    D, K, B = 3000, 32, 256
    eng = _engine(model, D, K, B, dtype, False)
    cells = np.random.default_rng(7).integers(0, 3000, 100)
    p0 = eng.params(registered_only=True)
    ref = None
    for rep in range(8):
        eng.set_params(p0)
        eng.reset_optimizer()
        eng.poison([0x00, 0xFF, 0x7F, 0x3C][rep % 4])
        out = eng.step(cells, 0.7, step_id=5)
        got = (out, eng.grads())
        if ref is None:
            ref = got
            continue
        assert got[0] == ref[0], (rep, got[0], ref[0])
        for k in ref[1]:
            assert np.array_equal(got[1][k], ref[1][k]), (rep, k)


def test_graph_recaptured_after_frozen_reload_fp8():
    """Reloading a frozen decoder weight changes the fp8 mode's power-of-two W_dec scale, a
    scalar the captured launch holds by value: the step graph must be re-captured (graph
    generation bumped by the repack), so graph and eager handles agree after the reload."""
    D, K, B = 3000, 32, 256
    cells = [np.random.default_rng(s).integers(0, 3000, B) for s in range(4)]
    res = []
    for graph in (False, True):
        eng = _engine("nb", D, K, B, "fp8", graph)
        out = [eng.step(cells[0], 1.0, step_id=1), eng.step(cells[1], 1.0, step_id=2)]
        name = "mu_dec.mu_decoding.weight"
        n = {k: v for k, v, _ in eng.param_info()}[name]
        eng.set_param(name, eng.get_param(name, n) * 8.0)  # amax x 8: wscale / 8
        out += [eng.step(cells[2], 1.0, step_id=3), eng.step(cells[3], 1.0, step_id=4)]
        res.append((out, eng.params(registered_only=True), eng.graph_stats()))
    assert res[1][2]["captures"] >= 4, res[1][2]  # two shapes' worth before and after the reload
    assert res[0][0] == res[1][0]
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[1][1][k]), k


@pytest.mark.parametrize("graph", [False, True])
def test_pipelined_steps_equal_synced_steps(graph):
    """Unsynced steps (the bench / training-loop pattern: the host stages step n + 1 into the other
    pinned slot while step n runs, and reuses a slot once the device has written back its staging
    ticket) must train exactly as steps synced one by one: a slot released too early would hand a
    later batch's cells to an earlier step.  Eval passes and bootstrap ridx interleave as in the
    reference loop (mmvae_alg.hh:277-311)."""
    D, K, B, N = 20000, 64, 1024, 20000
    rng = np.random.default_rng(3)
    plan = []
    for i in range(24):
        cells = rng.integers(0, N, B)
        if i % 4 == 0:
            plan.append(("eval", cells, None))
        else:
            plan.append(("step", cells, rng.integers(0, B, B)))
    res = []
    for sync in (True, False):
        from mmvae_amd import Engine
        eng = Engine(D=D, K=K, max_batch=B, dtype="bf16x3", seed=9)
        eng.synth_csr(N, lib_size=2000.0, seed=4)
        eng.init_params(seed=13)
        eng.graph(graph)
        for i, (kind, cells, ridx) in enumerate(plan):
            eng.run(cells, 0.7, ridx=ridx, update=kind == "step", step_id=500 + i, sync=sync)
        eng.sync()
        res.append(eng.params())
    for k in res[0]:
        assert np.array_equal(res[0][k], res[1][k]), k
