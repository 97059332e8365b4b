"""The RCCL gradient exchange on ONE GPU: a forced 1-rank communicator (-m gpu).

A communicator of one rank normally reduces nothing, so the engine skips the exchange at world 1.
MMVAE_FORCE_COMM=1 (read at mmvae_comm_init) keeps it on: the step then runs exactly the code a
world > 1 rank runs (capi.hip comm_bucket / enqueue_run) —

* the two overlapped buckets: split gradient kernels, an event fork onto the comm stream, one
  ncclGroupStart / ncclAllReduce-per-range / ncclGroupEnd per bucket, the join before clip + Adam;
* the flat path (the eager default; MMVAE_NO_OVERLAP=1 forces it): one ncclAllReduce of the whole
  gradient on the main stream;
* both inside a captured step graph (opt-in, MMVAE_COMM_GRAPH=1; the default runs them eagerly), after
  the ranks' capture agreement (comm_capture_agree: an eager ncclAllReduce(min) of the capture
  outcome) and, once, their agreement on the batch-dependent buffers' size (comm_sync_capacity);
* a capture that fails (MMVAE_TEST_COMM_CAPTURE_FAIL=1 makes comm_bucket refuse a capturing
  stream): the eager fallback for the handle's lifetime.

A sum over one rank is the identity, so every loss, clip norm, gradient and parameter must be
bit-identical to a handle without a communicator that runs the same split gradient kernels and
the k_sumsq clip norm (MMVAE_SPLIT_GRADS=1).  Reference step: mmvae_alg.hh:306-310 (backward,
clip_grad_norm_, Adam) with the all-reduce SURVEY §8(e) puts between backward and clip.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, K, B, N = 3000, 32, 384, 3000
MODES = {
    # name: (env at comm_init / steps, graph on, expect replays)
    "bucket": ({"MMVAE_OVERLAP": "1"}, False),
    "flat": ({}, False),  # (the default: eager steps, one flat all-reduce)
    "bucket_graph": ({"MMVAE_COMM_GRAPH": "1"}, True),
    "flat_graph": ({"MMVAE_COMM_GRAPH": "1", "MMVAE_NO_OVERLAP": "1"}, True),
    "capture_fail": ({"MMVAE_COMM_GRAPH": "1", "MMVAE_TEST_COMM_CAPTURE_FAIL": "1"}, True),
}


def _engine(model, dtype):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    eng = Engine(D=D, K=K, max_batch=B, dtype=dtype, seed=9, model=MODEL_VMF if model == "vmf" else MODEL_NB)
    eng.synth_csr(N, lib_size=1500.0, seed=4)
    eng.init_params(seed=13)
    if model == "vmf":
        eng.set_param("ln_kappa", np.array([np.log(np.float32(3.0))], np.float32))
    return eng


def _run(eng):
    """An update, an eval forward, three more updates (one ragged): the train loop's pattern."""
    out = []
    for s in range(5):
        cells = (np.arange(B, dtype=np.int64) * (7 + 2 * s) + 11 * s) % N
        if s == 1:
            out.append((eng.eval_loss(cells, 0.7, step_id=s), 0.0))
            continue
        if s == 4:
            cells = cells[:B - 40]
        out.append(eng.step(cells, 0.7, step_id=s))
    return out


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("model,dtype", [("nb", "bf16x3"), ("nb", "f32"), ("vmf", "bf16x3")])
def test_forced_one_rank_comm_bit_identical(model, dtype, mode, monkeypatch):
    from mmvae_amd import Engine
    env, graph = MODES[mode]
    # reference: no communicator, the same split gradient kernels and k_sumsq clip norm
    monkeypatch.setenv("MMVAE_SPLIT_GRADS", "1")
    ref = _engine(model, dtype)
    ref.graph(graph)
    want = _run(ref)
    want_p, want_g = ref.params(registered_only=True), ref.grads()
    ref.close()
    monkeypatch.delenv("MMVAE_SPLIT_GRADS")

    monkeypatch.setenv("MMVAE_FORCE_COMM", "1")
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    eng = _engine(model, dtype)
    eng.comm_init(0, 1, Engine.comm_unique_id())
    eng.graph(graph)
    got = _run(eng)
    st = eng.graph_stats()
    got_p, got_g = eng.params(registered_only=True), eng.grads()
    eng.close()

    assert got == want, (got, want)
    for k in want_p:
        assert np.array_equal(got_p[k], want_p[k]), k
        assert np.array_equal(got_g[k], want_g[k]), k
    if mode == "capture_fail":
        # the first update's capture failed: that step and every later one ran eagerly
        assert st["replays"] == 0 and st["captures"] == 0, st
    elif graph:
        # every run replayed a captured graph holding the RCCL calls (no eager fallback)
        assert st["replays"] == 5 and st["captures"] >= 3, st


def test_comm_graph_is_opt_in(monkeypatch):
    """Without MMVAE_COMM_GRAPH=1 (read at comm_init) a step with an active communicator runs
    eagerly even with step graphs enabled (captured collectives stay opt-in until a
    multi-rank run has exercised them)."""
    from mmvae_amd import Engine
    monkeypatch.setenv("MMVAE_FORCE_COMM", "1")
    monkeypatch.delenv("MMVAE_COMM_GRAPH", raising=False)
    eng = _engine("nb", "bf16x3")
    eng.comm_init(0, 1, Engine.comm_unique_id())
    eng.graph(True)
    _run(eng)
    st = eng.graph_stats()
    eng.close()
    assert st["replays"] == 0 and st["captures"] == 0, st


@pytest.mark.parametrize("streamed", [False, True])
def test_comm_graph_heavier_batch_keeps_its_graphs(streamed, monkeypatch):
    """a rank whose batch needs more entry-list (or streamed batch-set / DMA) room than it
    has seen used to re-allocate, re-capture and run the capture-agreement all-reduce alone while its
    peers replayed.  With step graphs holding RCCL calls the engine sizes those buffers once for every
    rank's worst batch (comm_sync_capacity), so a heavier batch replays the graphs already captured
    (one per staging slot) — and still matches a handle without a communicator bit for bit."""
    from mmvae_amd import Engine

    def make():
        eng = _engine("nb", "bf16x3")
        rp, col, val = eng.get_rows(np.arange(N, dtype=np.int64))
        if streamed:
            eng.stream_csr(rp, col, val)
        return eng, (rp, col, val)

    def run(eng, light, heavy):
        out = []
        for s in range(8):
            cells = heavy if s in (5, 6) else light
            out.append(eng.step(cells, 0.7, step_id=s))
        return out

    monkeypatch.setenv("MMVAE_SPLIT_GRADS", "1")
    ref, data = make()
    nnz = np.diff(data[0])
    order = np.argsort(nnz, kind="stable").astype(np.int64)
    light, heavy = order[:B].copy(), order[-B:].copy()
    assert nnz[heavy].sum() > 1.5 * nnz[light].sum()
    ref.graph(True)
    want = run(ref, light, heavy)
    want_p = ref.params(registered_only=True)
    ref.close()
    monkeypatch.delenv("MMVAE_SPLIT_GRADS")

    monkeypatch.setenv("MMVAE_FORCE_COMM", "1")
    monkeypatch.setenv("MMVAE_COMM_GRAPH", "1")  # (RCCL inside step graphs)
    eng, _ = make()
    eng.comm_init(0, 1, Engine.comm_unique_id())
    eng.graph(True)
    got = run(eng, light, heavy)
    st = eng.graph_stats()
    got_p = eng.params(registered_only=True)
    eng.close()
    assert got == want, (got, want)
    for k in want_p:
        assert np.array_equal(got_p[k], want_p[k]), k
    # one capture per staging slot for the single launch shape; the heavy batches replayed them
    assert st["captures"] == 2 and st["replays"] == 8, st


def test_comm_graph_uneven_slice_refused(monkeypatch):
    """With RCCL calls inside step graphs the key must follow from n_total (graph_key.hpp): a step
    whose B * world != n_total is refused before it issues any collective."""
    from mmvae_amd import Engine, MMVAEError
    monkeypatch.setenv("MMVAE_FORCE_COMM", "1")
    monkeypatch.setenv("MMVAE_COMM_GRAPH", "1")
    eng = _engine("nb", "bf16x3")
    eng.comm_init(0, 1, Engine.comm_unique_id())
    eng.graph(True)
    cells = np.arange(B, dtype=np.int64)
    with pytest.raises(MMVAEError):
        eng.step(cells, 0.7, n_total=B + 16, step_id=0)
    l, _ = eng.step(cells, 0.7, n_total=B, step_id=1)
    assert np.isfinite(l)
    eng.close()
