"""The engine's RCCL data-parallel step on two GPUs (-m gpu; skipped with fewer than 2 devices).

One spawned process per GPU, each touching the device only after the spawn. Ranks exchange the
128-byte RCCL id through a queue, call mmvae_comm_init and run world-2 mmvae_run(update=1) steps on
their shards (n_total = global batch, row_offset = shard start, so the Philox noise is keyed by the
global row). The result must equal a world-1 engine on the concatenated batch: per-step loss (sum of
the shards' loss), clip norm (of the all-reduced gradient), and the parameters after Adam. Run once
with the overlapped two-bucket exchange (capi.hip comm_bucket) and once with MMVAE_NO_OVERLAP=1 (one
all-reduce of the flat gradient). DESIGN.md §5.  Two ranks cannot share one device: RCCL 2.26 refuses
it in ncclCommInitRank ("invalid usage"), as checked on a one-GPU box of this pool.
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D, K, B, STEPS = 3000, 32, 512, 3


def _ndev():
    import torch
    return torch.cuda.device_count()


def _engine(model, b, device):
    from mmvae_amd import MODEL_NB, MODEL_VMF, Engine
    eng = Engine(D=D, K=K, max_batch=b, dtype="f32", seed=9, device=device,
                 model=MODEL_VMF if model == "vmf" else MODEL_NB)
    eng.synth_csr(3000, lib_size=1500.0, seed=4)
    eng.init_params(seed=13)
    if model == "vmf":
        eng.set_param("ln_kappa", np.array([np.log(np.float32(3.0))], np.float32))
    return eng


def _batches(skew=False, device=0):
    if not skew:
        return [(np.arange(B, dtype=np.int64) * (5 + 2 * s) + 3 * s) % 3000 for s in range(STEPS)]
    # rank 0's half from the lightest rows, rank 1's from the heaviest (only one rank's
    # batch outgrows the buffers it has seen): the synthetic dataset is the same in every process
    from mmvae_amd import MODEL_NB, Engine
    probe = Engine(D=D, K=K, max_batch=8, dtype="f32", seed=9, device=device, model=MODEL_NB)
    probe.synth_csr(3000, lib_size=1500.0, seed=4)
    rp, _, _ = probe.get_rows(np.arange(3000, dtype=np.int64))
    probe.close()
    order = np.argsort(np.diff(rp), kind="stable").astype(np.int64)
    h = B // 2
    return [np.concatenate([order[s * h:(s + 1) * h], order[3000 - (s + 1) * h:3000 - s * h]]) for s in range(STEPS)]


def _worker(rank, model, no_overlap, uid_q, res_q, device, graph=False, skew=False):
    try:
        # no_overlap: the flat all-reduce; otherwise the two buckets (the default with graphs;
        # forced by MMVAE_OVERLAP=1 for eager steps, whose default is flat)
        os.environ["MMVAE_NO_OVERLAP" if no_overlap else "MMVAE_OVERLAP"] = "1"
        if graph:  # RCCL calls inside step graphs are opt-in (read at comm_init)
            os.environ["MMVAE_COMM_GRAPH"] = "1"
        from mmvae_amd import Engine
        if rank == 0:
            uid = Engine.comm_unique_id()
            uid_q.put(uid)
        else:
            uid = uid_q.get(timeout=60)
        b = B // 2
        eng = _engine(model, b, device)
        eng.comm_init(rank, 2, uid)
        eng.graph(graph)  # the step graph then holds the RCCL bucket all-reduces
        out = []
        for s, cells in enumerate(_batches(skew, device)):
            l, n = eng.step(cells[rank * b:(rank + 1) * b], 0.7, n_total=B, row_offset=rank * b, step_id=s)
            out.append((l, n))
        if graph:
            out.append(eng.graph_stats())
        res_q.put((rank, out, eng.params(registered_only=True)))
    except Exception as ex:  # reported to the parent, which fails the test
        res_q.put((rank, "error", repr(ex)))


@pytest.mark.skipif(_ndev() < 2, reason="needs two GPUs (RCCL over xGMI)")
@pytest.mark.parametrize("no_overlap,graph,skew", [(False, False, False), (True, False, False), (False, True, False),
                                                   (False, True, True)])
@pytest.mark.parametrize("model", ["nb", "vmf"])
def test_rccl_world2_equals_world1(model, no_overlap, graph, skew):
    """skew: rank 1's shard holds the heaviest rows every step (its entry lists need more room than
    rank 0's), with the RCCL calls inside step graphs — every rank must still replay in step."""
    ctx = mp.get_context("spawn")
    uid_q, res_q = ctx.Queue(), ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, model, no_overlap, uid_q, res_q, r, graph, skew)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, out, params = res_q.get(timeout=110)
            assert out != "error", params
            res[r] = (out, params)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    if graph:  # every step replayed a captured graph (no eager fallback)
        for r in (0, 1):
            st = res[r][0].pop()
            assert st["replays"] == STEPS, st
    # world-1 reference in this process, on device 0
    full = _engine(model, B, 0)
    for s, cells in enumerate(_batches(skew)):
        l, n = full.step(cells, 0.7, step_id=s)
        l2 = res[0][0][s][0] + res[1][0][s][0]
        assert abs(l2 - l) <= 2e-5 * abs(l), (s, l2, l)
        for r in (0, 1):
            assert abs(res[r][0][s][1] - n) <= 2e-5 * n, (s, r, res[r][0][s][1], n)
    want = full.params(registered_only=True)
    for k, v in want.items():
        for r in (0, 1):
            got = res[r][1][k]
            err = float(np.max(np.abs(got - v)) / max(1e-30, float(np.max(np.abs(v)))))
            assert err <= 1e-5, (k, r, err)
