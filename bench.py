#!/usr/bin/env python
"""Benchmark: DSTAGNN_block forward+backward samples/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): one INNER DSTAGNN_block of the
PEMS08 geometry — B=32 per GPU, N=170, F=C=32, T=12, K=3, n_heads=3, d_model=512,
d_k=d_v=32, res_att (B,1,h,T,T) — train mode (both Dropout(0.05) on), random
make_model-style init, synthetic x ~ N(0,1), seeded d_out / d_re_At.
A step = forward + backward of one batch through the HIP library (+ the RCCL
all-reduce of the parameter gradients when --gpus > 1: data parallel, weak scaling).

Prints ONE JSON line (rank 0).  `roofline` is for the dominant kernel family, the GEMMs
(every dense contraction of the step: 27 gemm_f32 calls with their split-K folds): summed
algorithmic FLOP over summed durations, each call bracketed by HIP events on the stream it
runs on (dstagnn::prof_start/stop, serialised steps); `hot_kernel` keeps round 1's single
pre_conv forward GEMM figure; `hbm_roofline` is the metric's "%HBM roofline" (memory-side
bytes per step from the committed rocprofv3 PMC summary over this run's step time) with
the MFMA-busy fraction; `cpu_baseline` is the CPU oracle (a literal restatement of the
reference's loops, oracle/dstagnn_ref.py) timed on this host's cores on a bounded sample.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CFG = dict(B=32, N=170, T=12, K=3, n_heads=3, d_model=512, d_k=32, C=32)
PEAK_FP32_TFLOPS = 157.3   # MI355X dense fp32 (vector == f32 MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBS = 8000.0


def synth_graph(N, seed=0):
    rs = np.random.RandomState(seed)
    tmd = np.eye(N)
    pa = np.zeros((N, N))
    for i in range(N):
        tmd[i, rs.choice([j for j in range(N) if j != i], 2, replace=False)] = 1.0
        pa[i, rs.choice(N, 4, replace=False)] = 1.0
    return tmd, pa


def build_block(device):
    import dstagnn_drought_amd as D
    c = CFG
    tmd, pa = synth_graph(c["N"])
    Lt = D.scaled_Laplacian(torch.FloatTensor(tmd))
    cheb = [torch.from_numpy(p).float() for p in D.cheb_polynomial(Lt.numpy(), c["K"])]
    torch.manual_seed(1)
    blk = D.DSTAGNN_block("cpu", c["C"], c["C"], c["K"], c["C"], c["C"], 1, cheb, pa, tmd, c["N"], c["T"],
                          c["d_model"], c["d_k"], c["d_k"], c["n_heads"])
    for p in blk.parameters():  # make_model init (model/DSTAGNN_my.py:292-296)
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    D.set_direct_grads(blk)  # .grad written by the block's backward (no AccumulateGrad nodes)
    return blk.to(device).train(), cheb, torch.FloatTensor(pa)


def time_loop(step, steps, warmup):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def extras(dev, steps, warmup):
    """also the first block (F=1, res_att 0) and the full make_model train
    step (nb_block=4 as configurations/PEMS08_dstagnn.conf, SmoothL1 + Adam lr 1e-4)."""
    import dstagnn_drought_amd as D
    c = CFG
    B, N, T, K, h, Dm, dk, C = c["B"], c["N"], c["T"], c["K"], c["n_heads"], c["d_model"], c["d_k"], c["C"]
    tmd, pa = synth_graph(N)
    Lt = D.scaled_Laplacian(torch.FloatTensor(tmd))
    cheb = [torch.from_numpy(p).float() for p in D.cheb_polynomial(Lt.numpy(), K)]
    torch.manual_seed(1)
    blk = D.DSTAGNN_block("cpu", 1, 1, K, C, C, 1, cheb, pa, tmd, N, T, Dm, dk, dk, h)
    for p in blk.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
        else:
            torch.nn.init.uniform_(p)
    blk = D.set_direct_grads(blk.to(dev).train())
    gen = torch.Generator(device=dev).manual_seed(5)
    x1 = torch.randn(B, N, 1, T, device=dev, generator=gen)
    g1 = torch.randn(B, N, C, T, device=dev, generator=gen)
    g1r = torch.randn(B, 1, h, T, T, device=dev, generator=gen)
    prm = list(blk.parameters())

    def first_step():
        for p in prm:
            p.grad = None
        o, r = blk(x1, 0)
        torch.autograd.backward([o, r], [g1, g1r])
    t_first = time_loop(first_step, steps, warmup)

    net = D.make_model(dev, 1, 4, 1, K, C, C, 1, tmd, pa, tmd, T, T, N, Dm, dk, dk, h)
    D.set_direct_grads(net).train()
    from dstagnn_drought_amd.train import make_adam
    opt = make_adam(net.parameters(), 1e-4)
    crit = torch.nn.SmoothL1Loss().to(dev)
    xm = torch.randn(B, N, 1, T, device=dev, generator=gen)
    ym = torch.randn(B, N, T, device=dev, generator=gen)

    def model_step():
        opt.zero_grad(set_to_none=True)
        loss = crit(net(xm), ym)
        loss.backward()
        opt.step()
    t_model = time_loop(model_step, steps, warmup)
    return {"first_block": {"samples_per_s": round(B / t_first, 1), "ms_per_step": round(t_first * 1e3, 4),
                            "workload": "PEMS08 first DSTAGNN_block (F=1, res_att 0) fwd+bwd, B=32"},
            "model_step": {"samples_per_s": round(B / t_model, 1), "ms_per_step": round(t_model * 1e3, 4),
                           "workload": "make_model nb_block=4 PEMS08: fwd + SmoothL1 + bwd + Adam, B=32"}}


PMC_FILE = "profiles/block_pmc.json"


def load_pmc(stamp):
    """Counter summary of the same step (tools/pmc_step.sh -> tools/pmc_step_summary.py), or None;
    `stale` is set unless it was measured on this very library build (same libdstagnn.so sha)
    and workload."""
    try:
        with open(os.path.join(ROOT, PMC_FILE)) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    b = pmc.get("build") or {}
    pmc["stale"] = b.get("lib_sha256") != stamp["lib_sha256"] or pmc.get("workload", "pems08") != "pems08"
    return pmc


FAM_FILE = "profiles/family_rocprof.json"
PROF_KINDS = {0: "gemm_f32 (one call + split-K fold)", 1: "skinny_dw_kernel", 2: "tat_fused_fwd_kernel",
              3: "tat_fused_bwd_kernel", 4: "gtu_fwd_fused_kernel", 5: "gtu_bwd_fused_kernel", 6: "gtu_tconv_kernel",
              7: "sat_ln_bwd_fused_kernel"}


def dominant_kernel(recs, steps):
    """The single kernel (call site) with the most time per serialised step, from the per-call
    HIP-event records of dstagnn::prof_records ([kind, flops, bytes, ms] * n, in issue order; a
    call site = its position in the step): its own FLOP, bytes, duration and both roofline
    fractions (reported beside the family)."""
    groups = {}
    n_rec = len(recs) // 4
    per_step = max(1, n_rec // max(1, steps))  # the step's call sites in issue order (the same every step)
    for i in range(0, 4 * n_rec, 4):
        kind, fl, by, ms = int(recs[i]), recs[i + 1], recs[i + 2], recs[i + 3]
        key = (kind, (i // 4) % per_step)
        g = groups.setdefault(key, [0, 0.0, 0.0, 0.0])
        g[0] += 1
        g[1] += fl
        g[2] += by
        g[3] += ms
    if not groups:
        return None
    (kind, _), (n, fl, by, ms) = max(groups.items(), key=lambda kv: kv[1][3])
    tf = fl / (ms * 1e-3) / 1e12
    gbs = by / (ms * 1e-3) / 1e9
    return {"kernel": PROF_KINDS.get(kind, str(kind)), "launches_per_step": round(n / steps, 2),
            "avg_launch_us": round(ms / n * 1e3, 3), "gflop_per_launch": round(fl / n / 1e9, 4),
            "alg_mbytes_per_launch": round(by / n / 1e6, 3), "achieved_tflops": round(tf, 3),
            "mfma_frac": round(tf / PEAK_FP32_TFLOPS, 4), "achieved_GBs": round(gbs, 1),
            "hbm_frac": round(gbs / PEAK_HBM_GBS, 4),
            "bound": "mfma" if fl / max(by, 1.0) > PEAK_FP32_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9) else "hbm",
            "timing": "HIP events around each launch on its stream, serialised steps (dstagnn::prof_records)"}


def load_family_rocprof(stamp):
    """profiles/family_rocprof.json (tools/step_kernels.py --json) when it measured this build."""
    try:
        with open(os.path.join(ROOT, FAM_FILE)) as f:
            fr = json.load(f)
    except (OSError, ValueError):
        return None
    stale = (fr.get("build") or {}).get("lib_sha256") != stamp["lib_sha256"]
    fam = fr.get("family") or {}
    return {"file": FAM_FILE, "stale": stale, "achieved": None if stale else fam.get("achieved_tflops"),
            "frac": None if stale else fam.get("frac"), "us_per_step": fam.get("us"), "gflop_per_step": fam.get("gflop"),
            "kernels": fam.get("kernels"), "dominant_kernel": fr.get("dominant_kernel"), "build": fr.get("build")}


def algorithmic_flops_per_sample(c=CFG):
    """SURVEY.md §8(d) formula (sparse-T_k count, fwd; fwd+bwd = 3x)."""
    B, N, F, T, h, dk, D, K, C = 1, c["N"], c["C"], c["T"], c["n_heads"], c["d_k"], c["d_model"], c["K"], c["C"]
    nnzT = 4 * N
    fwd = 2 * (3 * F * T * N * h * dk + 2 * F * h * T * T * dk + F * T * h * dk * N + N * D * T * F
               + 2 * N * D * K * dk + K * N * N * dk + K * nnzT * F * T + K * N * T * F * C
               + sum(N * (T - k + 1) * 2 * C * C * k for k in (3, 5, 7)) + C * N * (3 * T - 12) * T)
    return 3 * fwd


def host_cores():
    """CPU share of this process: the GPU box exposes the whole machine in os.cpu_count()
    but grants ~16 cores per GPU (OMP_NUM_THREADS); use the smallest of the three."""
    n = os.cpu_count() or 1
    try:
        n = min(n, len(os.sched_getaffinity(0)))
    except AttributeError:
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, n)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(budget_s=12.0, warmup=2, min_iters=5, max_iters=20):
    """Oracle (literal restatement of the reference loops) on this host's cores, per BASELINE.md:
    `warmup` untimed iterations, then each fwd+bwd iteration timed on its own — at least
    `min_iters`, more while within `budget_s` — and the MEDIAN iteration reported."""
    from oracle import dstagnn_ref as ref
    c = CFG
    torch.set_num_threads(host_cores())
    threads = torch.get_num_threads()
    gen = torch.Generator().manual_seed(0)
    tmd, pa = synth_graph(c["N"])
    Lt = ref.scaled_laplacian(tmd)
    cheb = [torch.from_numpy(p).float() for p in ref.cheb_polynomials(Lt, c["K"])][:c["K"]]
    p = ref.random_block_params(gen, c["C"], c["C"], c["K"], c["C"], c["N"], c["T"], c["d_model"], c["d_k"], c["d_k"],
                                c["n_heads"])
    B = c["B"]
    x = torch.randn(B, c["N"], c["C"], c["T"], generator=gen)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], generator=gen)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], generator=gen)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], generator=gen)
    dims = dict(n_heads=c["n_heads"], d_k=c["d_k"], d_v=c["d_k"], K=c["K"])
    apa = torch.from_numpy(pa).float()
    for _ in range(warmup):
        ref.block_forward_backward(p, x, res, cheb, apa, dims, g_out, g_re, hoist=False)
    times, t0 = [], time.perf_counter()
    while len(times) < min_iters or (len(times) < max_iters and time.perf_counter() - t0 < budget_s):
        t1 = time.perf_counter()
        ref.block_forward_backward(p, x, res, cheb, apa, dims, g_out, g_re, hoist=False)
        times.append(time.perf_counter() - t1)
    med = float(np.median(times))
    return {"value": round(B / med, 3), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"median of {len(times)} timed fwd+bwd iterations (after {warmup} warm-ups) of the PEMS08 inner "
                      f"block at B={B} (oracle, literal T x K loop), {sum(times):.1f} s timed; "
                      f"min / max {B / max(times):.1f} / {B / min(times):.1f} samples/s"}


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(n):
    """`bench.py --gpus N` run without a launcher: start N ranks (one process per GPU) with
    torch.distributed.run on 127.0.0.1 and exit with its status.  Runs before anything
    touches the GPU (a child process, never an exec).  The same as the driver's own
    `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`
    (reference: xmp.spawn(main, nprocs=8), train_DSTAGNN_my.py:195-197)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    log(f"self-launch: {n} ranks via torch.distributed.run")
    return subprocess.call(cmd, env=env)


def init_ranks(gpus):
    """(rank, world, local) of this process; initialises the process group for world > 1.
    WORLD_SIZE (set by the launcher) must equal --gpus: a scaling run that silently measured
    another world size would be worse than a failure."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DSTAGNN_DIST_BACKEND=gloo + DSTAGNN_DEVICE_MOD=1 rehearse the multi-rank path on a single
    # GPU (ranks share cuda:0; RCCL refuses two ranks on one device) — test use only
    backend = os.environ.get("DSTAGNN_DIST_BACKEND", "nccl")
    local = local % int(os.environ.get("DSTAGNN_DEVICE_MOD", "1000000"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def launch_probe(rank, world):
    """--launch-probe: the launcher and the collective only (no GPU work; CPU tests run it
    over gloo): every rank contributes its rank, rank 0 prints what it saw."""
    t = torch.tensor([float(rank), 1.0])
    if world > 1:
        dist.all_reduce(t)
        dist.barrier()
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "ranks_seen": int(t[1]),
                          "rank_sum": int(t[0])}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hot-iters", type=int, default=50)
    ap.add_argument("--prof-steps", type=int, default=5, help="serialised steps for the GEMM-family event timing")
    ap.add_argument("--no-extras", action="store_true", help="skip the first-block / full-model lines")
    ap.add_argument("--launch-probe", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus))
    rank, world, local = init_ranks(args.gpus)
    if args.launch_probe:
        return launch_probe(rank, world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from dstagnn_drought_amd import _lib
    from dstagnn_drought_amd import block_fn as bf

    blk, cheb, apa = build_block(dev)
    c = CFG
    B = c["B"]
    gen = torch.Generator(device=dev).manual_seed(100 + rank)
    x = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=gen)
    res = torch.randn(B, 1, c["n_heads"], c["T"], c["T"], device=dev, generator=gen)
    g_out = torch.randn(B, c["N"], c["C"], c["T"], device=dev, generator=gen)
    g_re = torch.randn(B, c["C"], c["n_heads"], c["T"], c["T"], device=dev, generator=gen)
    params = [p for p in blk.parameters()]
    reducer = None
    if world > 1:
        from dstagnn_drought_amd.dp import GradAllReducer, mask_support_of
        reducer = GradAllReducer(blk.named_parameters(), mask_support=mask_support_of(blk)).attach(blk)

    def step():
        for p in params:
            p.grad = None
        out, re_at = blk(x, res)
        torch.autograd.backward([out, re_at], [g_out, g_re])
        if reducer is not None:  # the DP exchange step: bucketed RCCL all-reduce (mean)
            reducer.all_reduce()

    log(f"rank {rank}/{world}: block built, warmup {args.warmup}")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    t_issue = time.perf_counter() - t0  # host time to issue the steps (launch-bound if ~ elapsed)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    log(f"timed {args.steps} steps: {ms_per_step:.3f} ms/step (host issue {t_issue / args.steps * 1e3:.3f} ms/step)")
    value = world * B * args.steps / elapsed

    ops = _lib.load()
    names, ps, slots = blk._param_list()
    graph = blk._graph()
    sparse = bf.use_sparse(graph, blk.meta, c["T"])
    targs = (x, res, list(ps), slots, bf.graph_list(graph, sparse), bf.cfg_of(blk.meta), 0.05, 1,
             bf.flags_of(True, sparse, False))
    ops.block_time_stage(*targs, 10, 3)
    hot_ms = ops.block_time_stage(*targs, 10, args.hot_iters)

    # ---- dominant kernel family: the GEMMs (27 calls per step, the largest share of the step's
    # kernel time).  HIP event pairs around every GEMM call (kernel + split-K fold) over
    # --prof-steps steps run on ONE stream (dstagnn::prof_start serialises the block)
    fam = None
    if args.prof_steps > 0:
        ops.prof_start(4096)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.prof_steps):
            step()
        torch.cuda.synchronize()
        t_ser = (time.perf_counter() - t0) / args.prof_steps
        launches, flops, gbytes, gms, gmax, dropped = ops.prof_stop()
        P = args.prof_steps
        fam = dict(launches=launches / P, flops=flops / P, bytes=gbytes / P, ms=gms / P, max_ms=gmax,
                   serial_step_ms=t_ser * 1e3, dropped=dropped)
        dominant = dominant_kernel(ops.prof_records(), P)
    else:
        dominant = None
    stamp = _lib.build_stamp()
    pmc = load_pmc(stamp)
    rocprof_fam = load_family_rocprof(stamp)
    fresh = pmc is not None and not pmc["stale"]
    if fam is not None:
        achieved = fam["flops"] / (fam["ms"] * 1e-3) / 1e12
        roof = {"bound": "mfma", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                # bytes from the PMC summary only when it measured this build (else null + the
                # stale figure for reference)
                "traffic": pmc["gemm_family"]["bytes_corrected"] if fresh else None,
                "traffic_source": None if pmc is None else {"file": PMC_FILE, "stale": pmc["stale"],
                                                            "build": pmc.get("build")},
                "kernel": "gemm_f32 family: every GEMM call of one step (kernel + split-K fold), summed",
                "launches_per_step": round(fam["launches"], 1), "gflop_per_step": round(fam["flops"] / 1e9, 4),
                "ms_per_step": round(fam["ms"], 4), "avg_launch_us": round(fam["ms"] / fam["launches"] * 1e3, 3),
                "share_of_serial_step": round(fam["ms"] / fam["serial_step_ms"], 3),
                "min_bytes_per_step": int(fam["bytes"]),
                "timing": f"HIP events around each call, {args.prof_steps} serialised steps",
                # the same family from the committed rocprofv3 trace of a serialised step
                # (tools/step_trace.sh -> tools/step_kernels.py --json), when it measured this build
                "rocprof": rocprof_fam}
    else:
        roof = None
    # the single longest-running GEMM call site of round 1, kept for continuity: the pre_conv
    # forward GEMM (gemm_f32_hot_kernel), back-to-back launches timed with HIP events
    M, Nn, Kk = B * c["N"], c["d_model"], c["C"] * c["T"]
    hot_achieved = 2.0 * M * Nn * Kk / (hot_ms * 1e-3) / 1e12
    hot = {"kernel": "gemm_f32_hot_kernel (pre_conv fwd GEMM %dx%dx%d)" % (M, Nn, Kk),
           "avg_launch_us": round(hot_ms * 1e3, 3), "achieved": round(hot_achieved, 3), "unit": "TFLOP/s",
           "frac": round(hot_achieved / PEAK_FP32_TFLOPS, 4)}

    log(f"hot kernel {hot_ms * 1e3:.2f} us/launch")
    # opt-in bf16-operand GEMM variant (dstagnn::set_gemm_bf16): the same step, timed the same
    # way, reported beside the fp32 headline (never as `value`)
    bf16 = None
    if world == 1 and not args.no_extras:
        prev = ops.set_gemm_bf16(1)
        try:
            for _ in range(args.warmup):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            t_bf = (time.perf_counter() - t0) / args.steps
        finally:
            ops.set_gemm_bf16(prev)
        bf16 = {"ms_per_step": round(t_bf * 1e3, 4), "value": round(B / t_bf, 2), "unit": "samples/s",
                "dtype": "bf16 GEMM operands, fp32 accumulate / softmax / LayerNorm / reductions",
                "tolerance": "normwise ||err||/||ref|| <= 3e-2 per tensor vs the fp64 oracle "
                             "(tests/test_gpu_parity.py::test_bf16_gemm_variant)"}
        log(f"bf16 GEMM variant: {t_bf * 1e3:.3f} ms/step")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log(f"cpu baseline on {host_cores()} threads")
        cpu = cpu_baseline()
    ext = None
    if rank == 0 and world == 1 and not args.no_extras:
        log("extras: first block, full model step")
        ext = extras(dev, max(5, args.steps // 2), 3)
    # whole-block roofline: 758.8 MFLOP per sample fwd+bwd, compute-bound
    # (arithmetic intensity ~460 flop/B vs the fp32 ridge ~20): peak samples/s = 157.3 TF / F_alg
    # the metric's "%HBM roofline": memory-side bytes of one step (rocprofv3 FETCH_SIZE /
    # WRITE_SIZE passes, width-corrected: profiles/block_pmc.json) over this run's step time
    hbm_roof = None
    if pmc:
        bps = pmc["step"]["bytes_corrected"]
        gbs = bps / (ms_per_step * 1e-3) / 1e9
        hbm_roof = {"bytes_per_step": bps, "achieved_GBs": round(gbs, 1), "peak_GBs": PEAK_HBM_GBS,
                    "frac": round(gbs / PEAK_HBM_GBS, 4), "mfma_busy_frac": pmc["step"]["mfma_busy_frac"],
                    "gemm_mfma_busy_frac": pmc["gemm_family"]["mfma_busy_frac"], "source": PMC_FILE,
                    "stale": pmc["stale"], "pmc_build": pmc.get("build")}
        if pmc["stale"]:  # counters of another build: no fraction is claimed from them
            hbm_roof["frac"] = None
    f_alg = algorithmic_flops_per_sample()
    peak_sps = PEAK_FP32_TFLOPS * 1e12 / f_alg
    block_roof = {"bound": "mfma", "alg_flop_per_sample": round(f_alg / 1e6, 1), "unit_flop": "MFLOP",
                  "peak_samples_per_s_per_gpu": round(peak_sps, 0),
                  "frac": round(value / (world * peak_sps), 4)}

    if rank == 0:
        line = {
            "metric": "DSTAGNN_block fwd+bwd samples/sec (B,N=170,T=12) @1/2/4/8 GPU; %HBM roofline",
            "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
            "config": {"workload": "PEMS08 inner DSTAGNN_block fwd+bwd (train mode, dropout 0.05)",
                       "global_batch": B * world, "per_gpu_batch": B, "N": c["N"], "T": c["T"], "F": c["C"],
                       "K": c["K"], "n_heads": c["n_heads"], "d_model": c["d_model"], "d_k": c["d_k"],
                       "parallelism": f"dp{world}"},
            "algorithmic_tflops": round(algorithmic_flops_per_sample() * value / 1e12, 3),
            "roofline": roof,
            "dominant_kernel": dominant,
            "hot_kernel": hot,
            "block_roofline": block_roof,
            "hbm_roofline": hbm_roof,
            "cpu_baseline": cpu,
            "build": stamp,
        }
        if bf16 is not None:
            line["variant_bf16_gemm"] = bf16
        if ext is not None:
            line["extras"] = ext
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
