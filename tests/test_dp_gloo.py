"""Data-parallel decomposition on CPU with torch.distributed gloo, world size 2.

The engine's DP step (mm-vae_amd/csrc/capi.hip mmvae_run): each rank runs its
contiguous slice of the global batch with the loss divided by the GLOBAL batch, the registered
gradients are SUM all-reduced, then clip_grad_norm_ + Adam run redundantly on every rank.  Here
that step is executed on the oracle (oracle/nb_oracle.py NBTrainer.step_dp) with a real gloo
all-reduce and checked against the single-process reference step on the whole batch.
The batch split itself is the host helper mmvae_amd.shard_batch used by bench.py.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import sys

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (_ROOT, os.path.join(_ROOT, "mm-vae_amd", "py"), os.path.join(_ROOT, "tests")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from helpers import GOLDEN  # noqa: E402
import mmvae_amd  # noqa: E402
from oracle import nb_oracle, synth, vmf_oracle  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fixture(name="nb_mid.npz"):
    z = np.load(os.path.join(GOLDEN, name))
    init = {k[5:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("init/")}
    frozen = {k[7:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("frozen/")}
    return z, init, frozen


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    z, init, frozen = _fixture()
    D, B = int(z["D"]), int(z["B"])
    dp = nb_oracle.NBTrainer(init, frozen)
    ref = nb_oracle.NBTrainer(init, frozen)

    def allreduce(tensors):
        for t in tensors:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

    res = []
    for s in range(int(z["steps"])):
        cells = z[f"s{s}/cells"]
        # the global batch is the fixture's step batch; rank r takes rows [r B/W, (r+1) B/W)
        _, off = mmvae_amd.shard_batch(0, B, B, rank, world)
        rows = np.arange(off, off + B // world)
        x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells[rows], D))
        c = torch.from_numpy(z["covar"][cells[rows]])
        em = torch.from_numpy(z[f"s{s}/eps_mu"][rows])
        en = torch.from_numpy(z[f"s{s}/eps_nu"][rows])
        r = dp.step_dp(x, c, em, en, float(z[f"s{s}/beta"]), n_total=B, allreduce=allreduce)
        lt = torch.tensor([r["loss"]], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.SUM)
        # single-process reference step on the whole batch
        xa = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, D))
        ra = ref.step(xa, torch.from_numpy(z["covar"][cells]), torch.from_numpy(z[f"s{s}/eps_mu"]),
                      torch.from_numpy(z[f"s{s}/eps_nu"]), float(z[f"s{s}/beta"]))
        gerr = max(float((r["grads"][k] - ra["grads"][k]).abs().max() / (ra["grads"][k].abs().max() + 1e-30))
                   for k in ra["grads"])
        perr = max(float((dp.params()[k] - ref.params()[k]).abs().max()) for k in ra["grads"])
        # parameters must be bitwise identical across ranks after the update
        flat = torch.cat([v.reshape(-1) for v in dp.params().values()])
        other = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(other, flat)
        same = all(torch.equal(other[0], o) for o in other)
        res.append((float(lt.item()), ra["loss"], gerr, perr, r["total_norm"], ra["total_norm"], same))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_world2_matches_single_process():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    for rank in range(2):
        for (loss_dp, loss_ref, gerr, perr, n_dp, n_ref, same) in out[rank]:
            assert abs(loss_dp - loss_ref) <= 1e-5 * abs(loss_ref)
            assert gerr <= 1e-5, gerr
            assert abs(n_dp - n_ref) <= 1e-5 * n_ref
            assert perr <= 1e-6, perr
            assert same


def _vmf_worker(rank, world, port, out):
    """The vMF counterpart: loss over the global batch, the lbessel backward (Q3, independent
    of the upstream gradient) added on rank 0 only — as k_vgrad_small does under DP."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    z, init, frozen = _fixture("vmf_generic.npz")
    D, B = int(z["D"]), int(z["B"])
    dp = vmf_oracle.VMFTrainer(init, frozen)
    ref = vmf_oracle.VMFTrainer(init, frozen)

    def allreduce(tensors):
        for t in tensors:
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

    res = []
    for s in range(int(z["steps"])):
        cells = z[f"s{s}/cells"]
        _, off = mmvae_amd.shard_batch(0, B, B, rank, world)
        rows = np.arange(off, off + B // world)
        x = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells[rows], D))
        c = torch.from_numpy(z["covar"][cells[rows]])
        r = dp.step_dp(x, c, torch.from_numpy(z[f"s{s}/eps_mu"][rows]), float(z[f"s{s}/beta"]), n_total=B,
                       allreduce=allreduce, rank=rank)
        lt = torch.tensor([r["loss"]], dtype=torch.float64)
        dist.all_reduce(lt, op=dist.ReduceOp.SUM)
        xa = torch.from_numpy(synth.densify(z["rowptr"], z["col"], z["val"], cells, D))
        ra = ref.step(xa, torch.from_numpy(z["covar"][cells]), torch.from_numpy(z[f"s{s}/eps_mu"]),
                      float(z[f"s{s}/beta"]))
        gerr = max(float((r["grads"][k] - ra["grads"][k]).abs().max() / (ra["grads"][k].abs().max() + 1e-30))
                   for k in ra["grads"])
        perr = max(float((dp.params()[k] - ref.params()[k]).abs().max()) for k in ra["grads"])
        res.append((float(lt.item()), ra["loss"], gerr, perr, r["total_norm"], ra["total_norm"]))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_vmf_dp_world2_matches_single_process():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_vmf_worker, args=(2, port, out), nprocs=2, join=True)
    for rank in range(2):
        for (loss_dp, loss_ref, gerr, perr, n_dp, n_ref) in out[rank]:
            # the per-rank loss carries the kappa-only terms over its own rows: summed they are the
            # global batch's (fp32 constants of ~1e4 per cell: relative 1e-5)
            assert abs(loss_dp - loss_ref) <= 1e-5 * abs(loss_ref), (loss_dp, loss_ref)
            assert gerr <= 1e-4, gerr
            assert abs(n_dp - n_ref) <= 1e-5 * n_ref
            assert perr <= 1e-6, perr


def test_shard_batch_partitions_global_batch():
    N, B, W = 1000, 96, 4
    for batch in range(12):
        parts = [mmvae_amd.shard_batch(batch, B, N, r, W) for r in range(W)]
        ids = np.concatenate([p[0] for p in parts])
        # the union of the ranks' rows is exactly the reference's contiguous batch
        assert np.array_equal(ids, (batch * B + np.arange(B)) % N)
        assert [p[1] for p in parts] == [r * (B // W) for r in range(W)]
    with pytest.raises(ValueError):
        mmvae_amd.shard_batch(0, 10, N, 0, 3)
