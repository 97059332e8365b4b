#!/usr/bin/env python3
"""bench.py — NB-VAE ELBO-step throughput (cells/sec) on MI355X, BASELINE.json's metric.

One "step" = one reference ELBO step (include/mmvae_alg.hh:300-310): gather the batch's
cells from the HBM-resident CSR, forward, NB loss, backward, gradient all-reduce (N > 1),
clip_grad_norm_, Adam — all inside the HIP engine (mm-vae_amd/lib/libmmvae.so).
Workload (BASELINE configs[1]): synthetic 100k cells x 20k genes, latent 64, bf16 GEMM
operands, B = 4096 cells per GPU (weak scaling: global batch = 4096 N).

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line.  Inputs are resident in HBM before the timed region.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mm-vae_amd", "py"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md, chip-level parameters)
PEAK_HBM = 8.0e12            # B/s
PEAK_BF16 = 2.5e15           # dense MFMA flop/s
PEAK_F32_MFMA = 157.3e12
# vector ALU: 256 CU x 4 SIMD x 32 f32 lanes/clk x 2.4 GHz = 78.6e12 lane-ops/s; a
# transcendental (v_exp/v_log/v_rcp, quarter rate) counts as 4 lane-ops (MI355X_MICROARCH.md
# constants table: 8 vs 2 cycles per wave64 instruction)
PEAK_VALU = 256 * 4 * 32 * 2.4e9
# algorithmic VALU lane-ops per dense (cell, gene) element of the dominant kernel:
#   NB pass B: 6 transcendentals (softmax exp; softplus exp, log, rcp; 1/(nup s); log(s/nup)) x 4
#              + 36 f32 ops (mu, u, softplus/sigmoid/clamp, nup, s, q, loss, pq, du, 6 row/column
#              accumulations, bf16 convert) = 60
#   vMF decoder backward: exp x 4 + 9 f32 ops (covariate term, v, dv, column sums, dv*u, convert) = 13
VALU_PER_ELEM = {"nb": 60, "vmf": 13}
# dominant kernel per model: (name, GEMM flops per element / latent)
DOMINANT = {"nb": ("k_dec_nb", 6), "vmf": ("k_vdec_bwd", 4)}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="nb", choices=["nb", "vmf"])
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--genes", type=int, default=20000)
    ap.add_argument("--cells", type=int, default=100000)
    ap.add_argument("--latent", type=int, default=0, help="0 = 64 for NB (configs[1]), 32 for vMF (configs[2])")
    ap.add_argument("--lib-size", type=float, default=2000.0)
    ap.add_argument("--cpu-sample", type=int, default=1024)
    ap.add_argument("--cpu-steps", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--kernel-steps", type=int, default=5)
    return ap.parse_args()


def pmc_traffic(model, dtype, kernel):
    """HBM bytes per launch of `kernel` from the last committed rocprofv3 PMC passes
    (tools/pmc.sh -> profiles/pmc_traffic.json: (2 FETCH_SIZE + WRITE_SIZE) KiB, the gfx950
    FETCH_SIZE correction of MI355X_MICROARCH.md §HBM), or None if never profiled."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(f"{model}/{dtype}/{kernel}")
    except (OSError, ValueError):
        return None


def cpu_baseline(eng, args, Ncells):
    """The oracle (the reference's op sequence on ATen CPU fp32, oracle/nb_oracle.py) timed on
    this host: a bounded sample of the same workload (same dataset rows, same weights)."""
    import torch
    from oracle import nb_oracle, synth
    B = args.cpu_sample
    cells = np.arange(B) % Ncells
    rp, col, val = eng.get_rows(cells)
    x = torch.from_numpy(synth.densify(rp, col, val, np.arange(B), args.genes))
    c = torch.ones(B, 1)
    info = eng.param_info()
    P = {n: torch.from_numpy(eng.get_param(n, k)) for n, k, r in info if r}
    FR = {n: torch.from_numpy(eng.get_param(n, k)) for n, k, r in info if not r}
    g = torch.Generator().manual_seed(0)
    if args.model == "vmf":
        from oracle import vmf_oracle
        params, frozen = vmf_oracle.init_params(args.genes, Z=args.latent)
        params = {k: P[k].reshape(v.shape) for k, v in params.items()}
        frozen = {k: FR[k].reshape(v.shape) for k, v in frozen.items()}
        tr = vmf_oracle.VMFTrainer(params, frozen)

        def one():
            tr.step(x, c, torch.randn(B, args.latent, generator=g), 1.0)
    else:
        params, frozen = nb_oracle.init_params(args.genes, K=args.latent)
        params = {k: P[k].reshape(v.shape) for k, v in params.items()}
        frozen = {k: FR[k].reshape(v.shape) for k, v in frozen.items()}
        tr = nb_oracle.NBTrainer(params, frozen)

        def one():
            em = torch.randn(B, args.latent, generator=g)
            en = torch.randn(B, 1, generator=g)
            tr.step(x, c, em, en, 1.0)
    one()  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        one()
    dt = time.perf_counter() - t0
    return {"value": round(B * args.cpu_steps / dt, 2), "unit": "cells/sec", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{args.cpu_steps} {args.model.upper()} ELBO steps (fwd+bwd+clip+Adam) of B={B} cells of the same "
                      f"synthetic {args.genes}-gene dataset, K={args.latent}, fp32 ATen CPU "
                      f"({dt:.1f} s)"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    import mmvae_amd

    if args.latent == 0:
        args.latent = 32 if args.model == "vmf" else 64
    B, D, K, Ncells = args.batch, args.genes, args.latent, args.cells
    model = mmvae_amd.MODEL_VMF if args.model == "vmf" else mmvae_amd.MODEL_NB
    eng = mmvae_amd.Engine(D=D, K=K, max_batch=B, dtype=args.dtype, device=local, seed=1234, model=model)
    nnz = eng.synth_csr(Ncells, lib_size=args.lib_size, seed=2024)
    eng.init_params(seed=7)
    if world > 1:
        obj = [mmvae_amd.Engine.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        eng.comm_init(rank, world, obj[0])

    # weak scaling: B cells per rank, global batch B * world (mmvae_amd.shard_batch)
    batches = [mmvae_amd.shard_batch(s, B * world, Ncells, rank, world)[0] for s in range(args.warmup + args.steps)]
    beta = 1.0
    n_total = B * world

    def run(s):
        eng.run(batches[s], beta, update=True, n_total=n_total, row_offset=rank * B, step_id=s, sync=False)

    for s in range(args.warmup):
        run(s)
    eng.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.warmup, args.warmup + args.steps):
        run(s)
    eng.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    dt = t1 - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms = dt / args.steps * 1e3
    value = world * B * args.steps / dt

    # per-kernel device time (HIP events on the engine's stream), separate pass
    eng.timing(True)
    eng.timing_reset()
    for s in range(args.kernel_steps):
        run(s)
    eng.sync()
    tm = eng.timings()
    eng.timing(False)
    loss, _ = eng.run(batches[0], beta, update=False, n_total=n_total, row_offset=rank * B, step_id=0)

    if rank != 0:
        if world > 1:
            dist.barrier()
        return
    per_kernel = {k: v[0] / max(v[1], 1) for k, v in tm.items()}
    step_dev_ms = sum(v[0] for v in tm.values()) / args.kernel_steps
    dom, fpe = DOMINANT[args.model]
    t_dom = per_kernel[dom] * 1e-3
    lane_ops = float(VALU_PER_ELEM[args.model]) * B * D
    flops = float(fpe) * D * K * B
    achieved = lane_ops / t_dom
    # algorithmic HBM bytes of one launch: the batch's CSR entries (int32 gene + f32 count) +
    # the frozen decoder operands it streams once ([DP][KP] and, in the backward, [KP][DP])
    esz = 2 if args.dtype == "bf16" else 4
    alg_bytes = 8.0 * nnz / Ncells * B + 2 * ((D + 63) // 64 * 64) * (32 if K <= 32 else 64) * esz
    traffic = pmc_traffic(args.model, args.dtype, dom)
    # the dominant kernel is bound by the vector ALU, neither HBM nor MFMA: its
    # fraction of those two peaks is reported beside the VALU one
    roof = {"bound": "valu", "achieved": round(achieved / 1e12, 3), "peak": round(PEAK_VALU / 1e12, 3),
            "unit": "T f32 lane-ops/s (transcendental = 4)", "frac": round(achieved / PEAK_VALU, 4), "traffic": traffic,
            "kernel": dom, "kernel_ms": round(per_kernel[dom], 4),
            "hbm": {"algorithmic_bytes": alg_bytes, "achieved_gbs": round(alg_bytes / t_dom / 1e9, 1),
                    "peak_gbs": PEAK_HBM / 1e9, "frac": round(alg_bytes / t_dom / PEAK_HBM, 4)},
            "mfma": {"achieved_tflops": round(flops / t_dom / 1e12, 2),
                     "peak_tflops": (PEAK_BF16 if args.dtype == "bf16" else PEAK_F32_MFMA) / 1e12,
                     "frac": round(flops / t_dom / (PEAK_BF16 if args.dtype == "bf16" else PEAK_F32_MFMA), 4)}}
    out = {
        "metric": f"cells/sec (ELBO step) {'vMF' if args.model == 'vmf' else 'NB'}-VAE {D // 1000}k genes",
        "value": round(value, 1),
        "unit": "cells/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (seeded device-side generator, SURVEY §8(d) count distribution), random-init weights",
        "config": {"workload": f"{'vMF' if args.model == 'vmf' else 'NB'}-VAE ELBO step, {Ncells} cells x {D} genes, "
                               f"latent {K}, batch {B}/GPU",
                   "global_batch": B * world, "genes": D, "latent": K, "cells": Ncells,
                   "nnz_per_cell": round(nnz / Ncells, 1), "parallelism": f"dp{world}"},
        "roofline": roof,
        "device_ms_per_step": round(step_dev_ms, 4),
        "kernel_ms": {k: round(v, 4) for k, v in sorted(per_kernel.items(), key=lambda kv: -kv[1])},
        "eval_loss": loss,
    }
    if world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(eng, args, Ncells)
    print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()


if __name__ == "__main__":
    main()
