"""bench.py -- GFLOPS of C = A*A (CSR, FP64) on MI355X, the BASELINE.json metric.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--matrix NAME] [--no-cpu]

Workload (BASELINE.json configs[1]): cant.mtx A*A.  The real file is read from
$MHS_MATRIX_DIR/cant/cant.mtx when present; otherwise the synthetic cant-like
stand-in (mhspgemm.synth.cant_like: 62,451 rows, 27-point FEM stencil x 3 dof,
nnz(A*A) 17.5M vs the real 17.4M).  A "step" is one full SpGEMM: device-
resident A -> device-resident sorted C (mask formation, symbolic, numeric, C
allocation included: the t_e2e of BASELINE.md §2), C handed back to the
context's output pool after the step.

N = 1: one process.  N > 1: one rank per GPU over RCCL -- under torchrun (WORLD_SIZE set),
or, run bare as `python bench.py --gpus N`, bench.py starts the N ranks itself (child
processes, before any GPU call in the parent; --gpus above the visible GPU count is an
error, never a 1-GPU fallback).  Rows of A are
partitioned by flop, each rank starts with its row block of A (= of B); the
exchange plan is built once (mhspgemm.distributed.ShardPlan, outside the timed
steps) and a step is the exchange of B's rows over xGMI (--exchange halo: the
rows the block references; full: the north_star's allgatherv of every block)
+ the local SpGEMM; C stays distributed in `value`, and the gatherv of C to rank 0
is timed beside it (gather_C_ms, value_C_gathered; --no-gather skips it).  Total work is fixed, so scaling is "strong".

One JSON line on rank 0: value = 2*flop / (max over ranks of the time per step).
  roofline: the dominant kernel = the numeric phase (every numeric bin launch of a
            call: k_num_wave<10240,true> alone on this workload), timed with
            hipEvents recorded on the launch stream during the timed steps
            (MHS_OPT_NUMERIC_EVENTS).  achieved = COMPULSORY bytes of that phase
            per call / its average duration: read A once (row_ptr, col, val; B
            aliases A), read C's row_ptr, write C's col and val:
                B_comp = 8 (M+1) + 12 nnz(A) [+ B's arrays when B != A] + 12 nnz(C)
            traffic = measured HBM bytes of the same launches per call
            (rocprofv3 FETCH_SIZE*2 + WRITE_SIZE, separate --pmc passes, committed
            under profiles/ and keyed by matrix; null for a matrix never profiled).
            The old B_alg (12 B per product, as if every B gather missed to HBM)
            is kept only as the labelled "gather_equiv_GBps": it is not a bound.
  cpu_baseline: the oracle (CPU restatement, "port") on the same matrix, on the
            OpenMP threads the process gets (the GPU box grants 16 CPUs per GPU and
            sets OMP_NUM_THREADS=16, while nproc shows the whole host), median of repeats.
  configs:  (N = 1) the other BASELINE.json configs' stand-ins timed the same way
            (webbase-1M, mac_econ_fwd500, scircuit, cop20k_A, cage15, cant-perturbed;
            the metric's 16matrix.txt set, reference process.sh:21-37, printing
            src/main.cu:136): ms per step, GFLOPS, numeric ms and the compulsory-bytes
            fractions of the numeric phase and of the whole step.
  hbm_peak: (N = 1) measured copy / read / write bandwidth of the box
            (mhs_hbm_peak) beside the 8 TB/s spec the fractions are priced against.
  cold_call: one call on a fresh context (empty workspace and C pool: every
            hipMalloc inside, as the reference's Tool::allocate + C cudaMalloc,
            src/Tool.cu:4-45, src/main.cu:54-61) beside the pooled steady state.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for p in (str(ROOT), str(ROOT / "mh-spgemm_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

METRIC = json.loads((ROOT / "BASELINE.json").read_text())["metric"]
# numeric tiny classes (W lanes x K products per row; mirrors tiny_w / tiny_k of
# mh-spgemm_amd/csrc/mhs_internal.hpp): numeric bins NUM_TINY + c, c = 0..5
TINY_WK = [(4, 2), (8, 4), (16, 4), (32, 4), (64, 4), (64, 8)]
# numeric bin id -> kernel (mhs_internal.hpp NumBin; include/mhspgemm.h num_bins)
NUM_BIN_KERNELS = (["", "k_num_wave_direct<5120>", "k_num_wave_direct<10240>", "k_num_block<256>",
                    "k_num_block<1024>", "k_num_block<1024,global>", "k_num_wave<10240,grouped>",
                    "k_num_wave<10240,grouped> (up to 32 K products)"]
                   + [f"k_tiny_num_small({w}x{k}) (numeric-first rows: k_tiny_copy_rows)" if w <= 32
                      else f"k_tiny_num<{w},{k}>" for w, k in TINY_WK]
                   + ["k_num_wave_hash<5120>", "k_num_wave_hash<10240>"])
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# BASELINE.json configs[1..3] beyond the headline (configs[4]'s matrix at 1 GPU) + the perturbed cant
CONFIG_MATRICES = ["cant", "webbase-1M", "mac_econ_fwd500", "scircuit", "cop20k_A", "cage15", "cant-perturbed"]


def b_alg(M, nnzA, flop, nnzC):
    """Gather-equivalent bytes (12 B per product): a diagnostic, not a bound."""
    return 8 * (M + 1) + 20 * nnzA + 12 * flop + 12 * nnzC


def b_comp(M, nnzA, nnzC, nnzB_extra=0, MB_extra=0):
    """Compulsory bytes of C = A*B: A's arrays read once, C.ptr read, C.col/C.val
    written (B's arrays too when B does not alias A)."""
    return 8 * (M + 1) + 12 * nnzA + 12 * nnzC + 12 * nnzB_extra + 4 * MB_extra


# every kernel of the numeric phase: the bins' kernels and the numeric-first rows' slot copy
NUMERIC_PREFIXES = ("k_num_", "k_tiny_num", "k_tiny_copy")


def pmc_traffic(matrix: str):
    """Measured HBM bytes per call of the numeric launches of `matrix` from the
    committed rocprofv3 PMC summary (FETCH_SIZE doubled per the gfx950 correction,
    + WRITE_SIZE).  Returns (bytes, source, kernels) or (None, None, None)."""
    f = ROOT / "profiles" / "pmc_summary.json"
    try:
        d = json.loads(f.read_text())
        m = d["matrices"][matrix]
        ks = {k: v for k, v in m["kernels"].items()
              if k.split("::")[-1].startswith(NUMERIC_PREFIXES) and v.get("hbm_bytes_per_call") is not None}
        if not ks:
            return None, None, None
        tot = sum(v["hbm_bytes_per_call"] for v in ks.values())
        return float(tot), f"{m['source']} (head {d.get('head', '?')})", sorted(ks)
    except Exception:
        return None, None, None


def host_cpu():
    """(nproc, CPU model) of this host (the core count and lscpu model are stated)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        nproc = len(os.sched_getaffinity(0))
    except AttributeError:
        nproc = os.cpu_count() or 1
    return nproc, model


def cpu_baseline(A, budget_s: float = 12.0):
    """Oracle (C restatement of the reference path) on the same workload, on the
    threads OpenMP gives it; repeats until ~budget_s of CPU work, median."""
    from oracle import oracle as orc
    threads = orc.max_threads()
    times = []
    t_start = time.time()
    while True:
        t0 = time.perf_counter()
        orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N, nthreads=threads)
        times.append(time.perf_counter() - t0)
        if time.time() - t_start > budget_s or len(times) >= 50:
            break
    t1 = []  # one-thread figure, a single run
    t0 = time.perf_counter()
    orc.spgemm(A.ptr, A.col, A.val, A.ptr, A.col, A.val, A.N, nthreads=1)
    t1.append(time.perf_counter() - t0)
    return float(np.median(times)), threads, len(times), t1[0]


def check_gpus(n: int, backend: str, ndev: int) -> None:
    """--gpus N must name GPUs that exist (a gloo rehearsal may put every rank on one GPU)."""
    if n < 1:
        raise SystemExit(f"bench.py: --gpus {n}: needs at least one GPU")
    if backend != "gloo" and n > ndev:
        raise SystemExit(f"bench.py: --gpus {n} but only {ndev} GPU(s) visible (no silent 1-GPU fallback)")


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(cmd, n: int, poll_s: float = 0.2) -> int:
    """Start `cmd` as n child processes, one per rank (RANK = LOCAL_RANK = r, WORLD_SIZE = n,
    rendezvous on 127.0.0.1), wait for all of them and return the first non-zero exit code
    (the other ranks are then terminated: a dead rank would leave them in a collective).
    The parent never touches the GPU; rank 0's stdout (the JSON line) is inherited."""
    import subprocess
    port = str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, MHS_BENCH_LAUNCH="bench.py spawned its ranks", RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen(list(cmd), env=env))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                c = p.poll()
                if c is None:
                    continue
                live.remove(p)
                if c != 0 and rc == 0:
                    rc = c if c > 0 else 128 - c
                    for q in live:
                        q.terminate()
            if live:
                time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--matrix", default=None,
                    help="default: cant (BASELINE configs[1]) on 1 GPU, cage15 (configs[4], row-sharded) on N > 1")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-gather", action="store_true",
                    help="N>1: skip timing the gatherv of C to rank 0 (timed by default: SURVEY §8(e) asks for "
                         "the speed-up with C distributed and with C gathered)")
    ap.add_argument("--exchange", default="full", choices=["halo", "full"],
                    help="N>1: B rows moved per step: every row block (full: the north_star's allgatherv, "
                         "the headline) or only the referenced rows (halo); the other mode is timed beside it")
    ap.add_argument("--no-configs", action="store_true", help="N=1: skip the configs block")
    args = ap.parse_args()

    # MHS_BENCH_BACKEND=gloo: a rehearsal of the N > 1 path on a one-GPU box (every rank on
    # cuda:0, the exchange over gloo on host tensors) -- never a measurement
    backend = os.environ.get("MHS_BENCH_BACKEND", "nccl")
    import torch  # (importing torch and counting devices does not initialise the GPU)

    if "WORLD_SIZE" not in os.environ:
        check_gpus(args.gpus, backend, torch.cuda.device_count())
        if args.gpus > 1:
            # no launcher around us: start the N ranks ourselves, before any GPU call here
            sys.exit(spawn_ranks([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], args.gpus))

    import mhspgemm
    from mhspgemm import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}")
    if world > 1:
        check_gpus(world, backend, torch.cuda.device_count())
    N_GPUS = world
    if backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        dist_world = dist.get_world_size()
        if dist_world != world:
            raise SystemExit(f"bench.py: process group has {dist_world} ranks, WORLD_SIZE {world}")

    T_START = time.time()

    def log(msg):  # progress on stderr (rank 0): long N > 1 setups stay visible
        if rank == 0:
            print(f"[bench {time.time() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)

    if args.matrix is None:
        args.matrix = "cant" if world == 1 else "cage15"
    if world == 1:
        A, source = synth.load_or_synth(args.matrix)
        M_glob, nnzA = A.M, A.nnz
        flop = mhspgemm.flop_count_np(A.col, A.ptr)
    else:
        # one host copy per node: local rank 0 writes the matrix once as .npy files, every
        # rank memory-maps them and copies out only its row block (no rank holds a private
        # copy of the whole matrix)
        if local == 0:
            synth.build_shared(args.matrix)
        dist.barrier()
        M_glob, N_glob, s_ptr, s_col, s_val, source = synth.open_shared(args.matrix)
        log(f"{args.matrix}: {M_glob} rows, shared host copy ready")
        nnzA = int(s_ptr[-1])
        flop = mhspgemm.flop_count_np(s_col, s_ptr) if rank == 0 else 0
    tool = mhspgemm.Tool(local)
    tool.set_stream(torch.cuda.current_stream(local).cuda_stream)
    dev = f"cuda:{local}"
    xdev = "cpu" if backend == "gloo" else dev  # where the exchange's tensors live

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize(local)

    numeric_ms = []
    phases = []
    nnzC = 0
    gather_ms = None
    if world == 1:
        from mhspgemm import _lib as L

        def time_steps(A, steps, warmup):
            """Pipelined steps (no per-call host sync; hipEvents around each numeric phase on
            the launch stream).  Returns (elapsed s, numeric ms list)."""
            tool.set_option(L.MHS_OPT_SYNC, 0)
            tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, max(1, steps))
            for _ in range(warmup):
                C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
                C.release()
            barrier()
            t0 = time.perf_counter()
            for _ in range(steps):
                C, _ = mhspgemm.spgemm(tool, A, A, timing=False)
                C.release()
            barrier()
            el = time.perf_counter() - t0
            nms = tool.numeric_ms(steps)
            tool.set_option(L.MHS_OPT_SYNC, 1)
            tool.set_option(L.MHS_OPT_NUMERIC_EVENTS, 0)
            return el, nms

        A.H2D(local)
        elapsed, numeric_ms = time_steps(A, args.steps, args.warmup)
        t_max = elapsed
        # phase breakdown (reference Timing fields): separate, synchronised calls after
        # the timed region
        for _ in range(5):
            C, t = mhspgemm.spgemm(tool, A, A, timing=True)
            phases.append(t)
            C.release()
        nnzC = t.nnzC
        # cold call: a fresh context, so the workspace and C come from hipMalloc inside
        # the call (the pooled steps above reuse them)
        cold_tool = mhspgemm.Tool(local)
        cold_tool.set_stream(torch.cuda.current_stream(local).cuda_stream)
        C, tc = mhspgemm.spgemm(cold_tool, A, A, timing=True)
        C.release()
        cold_tool.close()
        cold = {"t_e2e_ms": round(tc.total_e2e, 4), "gflops": round(2.0 * flop / (tc.total_e2e * 1e-3) / 1e9, 2),
                "mem_alloc_ms": round(tc.mem_alloc, 4), "Malloc_C_col_val_ms": round(tc.Malloc_C_col_val, 4)}
        # the metric's set beyond the headline: every other 1-GPU BASELINE config stand-in,
        # timed exactly like the headline (fewer steps for the big ones)
        configs = []
        if not args.no_configs:
            for m in CONFIG_MATRICES:
                if m == args.matrix:
                    continue
                Am, src_m = synth.load_or_synth(m)
                fm = mhspgemm.flop_count_np(Am.col, Am.ptr)
                Am.H2D(local)
                st = max(3, min(args.steps, 10 if Am.M > 1_000_000 else args.steps))
                el, nms = time_steps(Am, st, max(1, min(args.warmup, 3)))  # >= 1: workspace growth untimed
                C, tm = mhspgemm.spgemm(tool, Am, Am, timing=True)
                C.release()
                ms = el / st * 1e3
                bcm = b_comp(Am.M, Am.nnz, tm.nnzC)
                avg_n = float(np.mean(nms))
                configs.append({
                    "matrix": m, "source": src_m, "rows": Am.M, "nnzA": Am.nnz, "flop": fm, "nnzC": tm.nnzC,
                    "steps": st, "ms_per_step": round(ms, 4), "gflops": round(2.0 * fm / (ms * 1e-3) / 1e9, 2),
                    "numeric_ms": round(avg_n, 4), "compulsory_bytes": bcm,
                    "frac_numeric": round(bcm / (avg_n * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                    "frac_e2e": round(bcm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                    "_frac_e2e": bcm / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS,
                    "suitesparse_stats": synth.TARGETS.get(m),
                    # the stand-in's deviation from them (say how close each stand-in is)
                    "standin_vs_suitesparse": ({k: round(synth.ACHIEVED[m][k] / v - 1, 3)
                                                for k, v in synth.TARGETS[m].items() if k in synth.ACHIEVED.get(m, {})}
                                               if src_m.startswith("synthetic") and m in synth.TARGETS else None),
                    "phases_ms": {k: round(getattr(tm, k), 4) for k in (
                        "Form_mask_matrix_B", "symbolic_binning", "Calculate_C_nnz", "numeric_binning", "Numeric",
                        "total_e2e")},
                })
                log(f"config {m}: {ms:.3f} ms per step, {configs[-1]['gflops']} GFLOPS")
                Am.d_release_csr()
                del Am
            tool.release()
        try:
            hbm = tool.hbm_peak(2 << 30, 10)
        except Exception as e:  # a diagnostic: never fails the bench
            hbm = {"error": str(e)}
    else:
        from mhspgemm import distributed as D
        from mhspgemm import _lib as L
        # the same matrix on ONE GPU first (rank 0, the other ranks wait): the speed-up of
        # this line is computed on one workload
        one_gpu = None
        if rank == 0:
            A1 = mhspgemm.CSR(M_glob, N_glob, np.array(s_ptr), np.array(s_col), np.array(s_val))
            A1.H2D(local)
            t1 = mhspgemm.Tool(local)
            t1.set_stream(torch.cuda.current_stream(local).cuda_stream)
            t1.set_option(L.MHS_OPT_SYNC, 0)
            for _ in range(args.warmup):
                C, _ = mhspgemm.spgemm(t1, A1, A1, timing=False)
                C.release()
            torch.cuda.synchronize(local)
            t0 = time.perf_counter()
            for _ in range(args.steps):
                C, _ = mhspgemm.spgemm(t1, A1, A1, timing=False)
                C.release()
            torch.cuda.synchronize(local)
            ms1 = (time.perf_counter() - t0) / args.steps * 1e3
            one_gpu = {"ms_per_step": round(ms1, 4), "value": round(2.0 * flop / (ms1 * 1e-3) / 1e9, 2),
                       "note": "the same matrix, whole, on rank 0's GPU alone (same steps / warmup)"}
            log(f"one-GPU leg: {ms1:.3f} ms per step")
            t1.close()
            A1.release()
            del A1
            torch.cuda.empty_cache()
        barrier()
        tool.set_option(L.MHS_OPT_SYNC, 0)  # stream-ordered calls: no host wait after the numeric launch
        # each rank keeps only its equal-row block of the input (what a rank reading its part
        # of the file would hold); the flop balance and the exchange plan are built from the
        # blocks with collectives, timed as plan_ms (setup, outside the steps)
        r0, r1 = D.equal_rows(M_glob, world, rank)
        eq = D.local_block(s_ptr, s_col, s_val, r0, r1, xdev)
        del s_col, s_val
        barrier()
        p0 = time.perf_counter()
        blk = D.rebalance(eq, M_glob, compute=dev)  # (rehearsal: host block, GPU gathers)
        del eq
        plan = D.ShardPlan(blk, M_glob, mode=args.exchange)
        barrier()
        plan_ms = (time.perf_counter() - p0) * 1e3
        log(f"plan built in {plan_ms:.0f} ms")
        mult = D.hip_local_multiply(tool)
        if xdev != dev:  # rehearsal: the exchanged rows go to the GPU for the HIP multiply
            hip_mult = mult

            def mult(A, Bp, Bc, Bv, N):
                Ag = D.Block(A.r0, A.r1, A.ptr.to(dev), A.col.to(dev), A.val.to(dev))
                return hip_mult(Ag, Bp.to(dev), Bc.to(dev), Bv.to(dev), N)

        def timed(pl):
            for _ in range(args.warmup):
                C, _ = D.spgemm_planned(pl, mult)
                C.release()
            barrier()
            t0 = time.perf_counter()
            nloc = 0
            for _ in range(args.steps):
                C, _ = D.spgemm_planned(pl, mult)
                nloc = C.nnz
                C.release()
            barrier()
            tt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=xdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            nn = torch.tensor([nloc, pl.bytes_in, pl.nB], dtype=torch.int64, device=xdev)
            dist.all_reduce(nn)
            return float(tt.item()), [int(x) for x in nn.tolist()]

        t_max, (nnzC, xbytes, xrows) = timed(plan)
        log(f"{args.exchange} steps: {t_max / args.steps * 1e3:.3f} ms per step")
        # the other exchange mode beside it (the north_star's allgatherv when the headline is halo)
        alt_mode = "full" if args.exchange == "halo" else "halo"
        alt_plan = D.ShardPlan(blk, M_glob, mode=alt_mode)
        t_alt, (_, alt_bytes, _) = timed(alt_plan)
        del alt_plan
        if not args.no_gather:
            # gatherv of C's row blocks to rank 0 (the speed-up is reported with C
            # distributed and with C gathered); median of 3, max over ranks
            tool.set_option(L.MHS_OPT_SYNC, 1)
            C, _ = D.spgemm_planned(plan, mult)
            Cs = C if xdev == dev else tuple(x.cpu() for x in C.to_torch())
            gt = []
            for _ in range(3):
                barrier()
                g0 = time.perf_counter()
                g = D.gather_result(Cs, blk)
                barrier()
                gt.append((time.perf_counter() - g0) * 1e3)
                del g
            tt = torch.tensor([float(np.median(gt))], dtype=torch.float64, device=xdev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            gather_ms = float(tt.item())
            del Cs
            C.release()
            log(f"gatherv(C) to rank 0: {gather_ms:.3f} ms")

    ms_per_step = t_max / args.steps * 1e3
    gflops = 2.0 * flop / (ms_per_step * 1e-3) / 1e9
    if rank != 0:
        if dist is not None:
            dist.barrier()
            dist.destroy_process_group()
        return

    balg = b_alg(M_glob, nnzA, flop, nnzC)
    out = {
        "metric": METRIC,
        "value": round(gflops, 2),
        "unit": "GFLOPS",
        "n_gpus": N_GPUS,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic" if source.startswith("synthetic") else "file",
        "config": {
            "workload": f"{args.matrix}.mtx A*A ({source}), device-resident A -> device-resident sorted C",
            "matrix": args.matrix, "rows": M_glob, "nnzA": nnzA, "flop": flop, "nnzC": nnzC,
            "parallelism": "single GPU" if N_GPUS == 1 else
                           f"row-sharded x{N_GPUS}, {'full allgatherv (north_star)' if args.exchange == 'full' else 'halo'} "
                           f"exchange of B's rows in every step (value), {'halo' if args.exchange == 'full' else 'full allgatherv'} "
                           f"beside it (exchange_alt), C distributed"
                           + (" [gloo rehearsal on one GPU: not a measurement]" if backend == "gloo" else ""),
            "memory": "steady-state steps reuse the context's workspace and pooled C buffers "
                      "(no hipMalloc in a step); cold_call times a fresh context",
        },
    }
    if N_GPUS == 1:
        avg_num = float(np.mean(numeric_ms))
        bc = b_comp(M_glob, nnzA, nnzC)
        achieved = bc / (avg_num * 1e-3) / 1e9
        traffic, tsrc, tkern = pmc_traffic(args.matrix)
        nk = [k for k, c in zip(NUM_BIN_KERNELS, phases[-1].num_bins) if c > 0 and k]
        out["roofline"] = {
            "bound": "hbm", "kernel": "numeric phase: " + ", ".join(nk),
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": traffic, "traffic_source": tsrc, "traffic_kernels": tkern,
            "bytes_per_launch": bc, "bytes_definition": "compulsory: 8(M+1) + 12 nnz(A) + 12 nnz(C)",
            "avg_launch_ms": round(avg_num, 4),
            "hbm_measured_GBps": round(traffic / (avg_num * 1e-3) / 1e9, 1) if traffic else None,
            "frac_measured": round(traffic / (avg_num * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4) if traffic else None,
            "e2e_frac": round(bc / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
            "gather_equiv_GBps": round(balg / (ms_per_step * 1e-3) / 1e9, 1),
        }
        assert out["roofline"]["frac"] <= 1.0 and out["roofline"]["e2e_frac"] <= 1.0, out["roofline"]
        out["cold_call"] = cold
        if "copy_GBps" in hbm:
            out["roofline"]["peak_measured_copy"] = hbm["copy_GBps"]
            out["roofline"]["frac_vs_measured_copy"] = round(achieved / hbm["copy_GBps"], 4)
            #  the launch priced against the measured read and write peaks for its
            # own mix: compulsory reads (A's arrays, C.ptr) at the read peak plus compulsory writes
            # (C.col / C.val) at the write peak, over its measured duration
            rd, wr = 8 * (M_glob + 1) + 12 * nnzA, 12 * nnzC
            if hbm.get("read_GBps") and hbm.get("write_GBps"):
                t_ideal = rd / (hbm["read_GBps"] * 1e9) + wr / (hbm["write_GBps"] * 1e9)
                out["roofline"]["frac_vs_measured_read_write"] = round(t_ideal / (avg_num * 1e-3), 4)
        out["hbm_peak"] = dict(hbm, spec_GBps=HBM_PEAK_GBPS,
                               kernels="mhs_hbm_peak: the best of 38 kernel shapes per kind (16 B a lane, 2-16 accesses in flight, grid-stride or one slab per block, 1-32 blocks per CU, cached or nontemporal) and the runtime's own D2D copy / fill, 2 GiB buffers")
        if configs:
            fr = [c.pop("_frac_e2e") for c in configs]  # unrounded
            fr.append(b_comp(M_glob, nnzA, nnzC) / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBPS)
            geo = float(np.exp(np.mean(np.log(fr))))
            out["configs"] = {"matrices": configs, "geomean_frac_e2e_with_headline": round(geo, 4),
                              "note": "same pipelined steps as value; frac_* = compulsory bytes "
                                      "8(M+1) + 12 nnz(A) + 12 nnz(C) over the numeric phase / the whole step, "
                                      "vs the 8 TB/s spec"}
        ph = {k: round(float(np.mean([getattr(p, k) for p in phases])), 4)
              for k in ("mem_alloc", "Form_mask_matrix_B", "symbolic_binning", "Calculate_C_nnz",
                        "numeric_binning", "Malloc_C_col_val", "Numeric", "total_e2e")}
        ph["t_ref_getTotal"] = round(float(np.mean([p.getTotal() for p in phases])), 4)
        ph["note"] = "5 synchronised calls with per-phase events, after the timed region"
        out["phases_ms"] = ph
        out["bins"] = {"symbolic": phases[-1].sym_bins[:12], "numeric": phases[-1].num_bins[:16],
                       "numeric_kernels": {NUM_BIN_KERNELS[i]: c for i, c in enumerate(phases[-1].num_bins[:16])
                                           if i and c}}
        if not args.no_cpu:
            med, threads, reps, one = cpu_baseline(A)
            nproc, model = host_cpu()
            out["cpu_baseline"] = {
                "value": round(2.0 * flop / med / 1e9, 3), "unit": "GFLOPS", "cores": threads,
                "kind": "port",
                "sample": f"full {args.matrix} A*A (symbolic+numeric, Gustavson, oracle/), median of {reps} "
                          f"runs of {med*1e3:.1f} ms on {threads} OpenMP threads; 1 thread: "
                          f"{2.0 * flop / one / 1e9:.3f} GFLOPS ({one*1e3:.0f} ms)",
                "host": {"nproc": nproc, "cpu_model": model, "omp_threads": threads,
                         "cap": "OMP_NUM_THREADS: the GPU box grants 16 CPUs per GPU (harness setting); "
                                "nproc counts the whole host"},
            }
        else:
            out["cpu_baseline"] = None
    else:
        out["roofline"] = None
        out["cpu_baseline"] = None
        out["exchange"] = {"mode": args.exchange, "bytes_in_per_step_all_ranks": xbytes,
                           "local_B_rows_all_ranks": xrows, "plan_ms": round(plan_ms, 3),
                           "plan": "distributed flop balance from equal-row blocks (mhspgemm.distributed.rebalance) "
                                   "+ ShardPlan, collectives only, timed once before the steps"}
        ms_alt = t_alt / args.steps * 1e3
        out["exchange_alt"] = {"mode": alt_mode, "value": round(2.0 * flop / (ms_alt * 1e-3) / 1e9, 2),
                               "ms_per_step": round(ms_alt, 4), "bytes_in_per_step_all_ranks": alt_bytes}
        out["dist_backend"] = dist.get_backend()
        out["rccl_world_size"] = dist_world if backend != "gloo" else None
        out["launch"] = os.environ.get("MHS_BENCH_LAUNCH", "external launcher (WORLD_SIZE set)")
        out["single_gpu_same_matrix"] = one_gpu
        out["speedup_vs_1gpu"] = round(one_gpu["ms_per_step"] / ms_per_step, 3)
        if gather_ms is not None:
            out["gather_C_ms"] = round(gather_ms, 3)
            out["speedup_vs_1gpu_C_gathered"] = round(one_gpu["ms_per_step"] / (ms_per_step + gather_ms), 3)
            out["value_C_gathered"] = round(2.0 * flop / ((ms_per_step + gather_ms) * 1e-3) / 1e9, 2)
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
