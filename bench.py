"""bench.py -- full RMT time step (soft disc in the lid-driven cavity, configs 2/4
physics) on MI355X: cell-updates/s at N=4096 (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n 4096] [--no-cpu-baseline]
                  [--config 4|2|3|5]

--config names a BASELINE.json configuration (default 4, the one the metric is quoted on):
  2  soft_disc_in_lid_driven N=256 semilagrangian        (208 B/cell)
  3  disc_in_taylor_green N=1024 WENO5 + SSP-RK3          (224 B/cell)
  4  soft_disc_in_lid_driven N=4096 semilagrangian       (208 B/cell)
  5  mac_multi_disc_lid N=8192, 3 discs (seed 3)          (280 B/cell)
Configs 2/3/5 are single-GPU lines for the per-config roofline (the driver's line is config 4).

A step is one loop body of benchmarks/soft_disc_in_lid_driven.py:206-235 (timestep,
reference-map advection, narrow-band extrapolation, level-set rebuild, RK4 momentum,
Rhie-Chow + DCT-I projection, centroid/J diagnostics) on synthetic state of that shape
(the driver's own initial condition: disc (0.6, 0.5, 0.2), fluid at rest, lid U=1).

Multi-GPU (--gpus N > 1, one process per GPU under torch.distributed.run): the SAME
N=4096 problem decomposed into N row slabs (pyrmt_amd/distributed.py, librmt rmt_slab_*),
RCCL halo exchanges / all-to-all transposes / allgathers over xGMI -- strong scaling;
`value` = the problem's cell-updates per second, timed by the max over ranks.
"""
import argparse
import json
import os
import platform
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# algorithmic fp64 plane traffic of the stress + 4-stage RK4 pass
# (reads u, v, p, X1, X2; writes u*, v*) = 7 planes x 8 B per cell for one RK4 pass.
RK4_ALG_BYTES_PER_CELL = 7 * 8
STEP_ALG_BYTES_PER_CELL = 208  # the whole step
# per BASELINE config: (grid, algorithmic bytes per cell-update of the whole step, workload)
CONFIGS = {
    2: (256, 208, "soft_disc_in_lid_driven N=256 semilagrangian (config 2)"),
    3: (1024, 224, "disc_in_taylor_green N=1024 weno5 + SSP-RK3 (config 3)"),
    4: (4096, 208, "soft_disc_in_lid_driven N=4096 semilagrangian (configs 2/4 loop body)"),
    5: (8192, 280, "mac_multi_disc_lid N=8192, 3 discs, seed 3 (config 5)"),
}
# HBM bytes per launch and per step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this
# bench (scripts/r06_evidence.sh -> tools/pmc_traffic.py; FETCH x2 per the gfx950 calibration)
PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r06", "ev", "pmc_traffic_n4096.json")
# the same passes for the config-3 / config-5 lines (scripts/r06_evidence.sh OUT 53)
PMC_TRAFFIC_CFG = {3: os.path.join(ROOT, "profiles", "r06", "ev", "pmc_traffic_cfg3_n1024.json"),
                   5: os.path.join(ROOT, "profiles", "r06", "ev", "pmc_traffic_cfg5_n8192.json")}
# fp64 VALU counts of the same kernel and the measured FMA peak (scripts/pmc_f64.sh ->
# tools/f64_roof.py): k_mom_stage is VALU-issue-bound, not HBM-bound
F64_ROOF = os.path.join(ROOT, "profiles", "r06", "ev", "f64_roof_n4096.json")
# dependency depth of the bench-state extrapolation chain at N=4096: the longest sequence of
# fits each reading the previous one (tools/chain_dag_depth.py over the exact DAG)
CHAIN_DAG = os.path.join(ROOT, "profiles", "r05", "chain_dag_n4096.json")


def _chain_depth(n):
    if n != 4096 or not os.path.exists(CHAIN_DAG):
        return None
    return json.load(open(CHAIN_DAG))["depth"]
# the reference's only published timing: the collocated soft-disc step at N=128 on "CPU
# (8 threads)", ~31 ms/step (docs/PERFORMANCE.md:3-5) = 0.53 M cell-updates/s
REF_PUBLISHED = {"value": 128 * 128 / 0.031, "unit": "cell-updates/s", "grid": 128,
                 "ms_per_step": 31.0, "source": "reference docs/PERFORMANCE.md:3-5 (CPU, 8 threads)"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def _pmc(n, ws):
    """(bytes per k_mom_stage launch, bytes per step, git rev) from the committed PMC passes."""
    if n != 4096 or ws != 1 or not os.path.exists(PMC_TRAFFIC):
        return None, None, None
    d = json.load(open(PMC_TRAFFIC))
    k = d["kernels"].get("k_mom_stage")     # the full-grid stage launches the events time
    return (k["bytes_per_full_launch"] if k else None), d["per_step"].get("total"), d.get("git_rev")


def _f64_roof(n, ws, launch_s):
    """k_mom_stage against its fp64 VALU roof (committed counter pass), or None."""
    if n != 4096 or ws != 1 or not os.path.exists(F64_ROOF):
        return None
    d = json.load(open(F64_ROOF))
    achieved = d["flop_per_launch"] / launch_s / 1e12
    return {"bound": "valu-f64", "kernel": d["kernel"], "achieved": achieved,
            "peak": d["fma_peak_tflops_measured"], "unit": "TFLOP/s",
            "frac": achieved / d["fma_peak_tflops_measured"],
            "issue_floor_ms": d["valu_issue_floor_ms"],
            "issue_frac": d["valu_issue_floor_ms"] / (launch_s * 1e3),
            "counters_rev": d["git_rev"]}


def _dist():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def cpu_baseline(n, steps):
    """The oracle (C restatement of the reference's Numba kernels + the same NumPy/SciPy
    calls) timed on this host, two ways: faithful threading (OpenMP only in the kernels the
    reference runs Numba parallel=True; everything else serial, as the reference) and
    all-cores (OpenMP on every per-cell loop; the extrapolation sweep stays serial).  Both
    give the same results bit for bit.  Threads: the box's CPU share (16), os.cpu_count()
    reports the whole machine there."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    cores = min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 16)
    O.set_threads(cores)
    out = {}
    for mode, allc in (("faithful", False), ("all_cores", True)):
        O.set_all_cores(allc)
        sim = O.SoftDisc(n, "lid")
        t0 = time.perf_counter()
        for _ in range(steps):
            sim.step()
        dt = time.perf_counter() - t0
        out[mode] = {"value": n * n * steps / dt, "s_per_step": dt / steps}
    O.set_all_cores(False)
    f = out["faithful"]
    return {"value": f["value"], "unit": "cell-updates/s", "cores": cores, "kind": "port",
            "all_cores": {"value": out["all_cores"]["value"],
                          "s_per_step": out["all_cores"]["s_per_step"], "cores": cores},
            "cpu": _cpu_model(), "nproc": os.cpu_count(),
            "reference_published": REF_PUBLISHED,
            "sample": f"{steps} full step(s) of the N={n} soft-disc loop body per variant "
                      f"(oracle: faithful {f['s_per_step']:.1f} s/step with OpenMP only where "
                      f"the reference uses Numba parallel=True; all-cores "
                      f"{out['all_cores']['s_per_step']:.1f} s/step) on {_cpu_model()}"}


def cpu_baseline_cfg(cfg, n):
    """Configs 3 and 5: the oracle on a bounded sample of the same loop (config 5's N=8192 MAC
    step takes ~90 s in the oracle: the sample is one step at N=2048, per cell-update)."""
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    cores = min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else 16)
    O.set_threads(cores)
    O.set_all_cores(True)
    if cfg == 3:
        sim, m, steps, rec = O.SoftDisc(n, "tg", "weno5"), n, 2, {"energies": True}
    else:
        from oracle import mac_oracle as M
        m = 2048
        sim, steps, rec = M.MacMultiDisc(m), 1, {}
    t0 = time.perf_counter()
    for _ in range(steps):
        sim.step(**rec)
    dt = time.perf_counter() - t0
    O.set_all_cores(False)
    return {"value": m * m * steps / dt, "unit": "cell-updates/s", "cores": cores, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"{steps} step(s) of the config-{cfg} loop at N={m} (oracle, all-cores "
                      f"OpenMP, {dt / steps:.1f} s/step) on {_cpu_model()}"}


def main_config(args, cfg):
    """One single-GPU line for BASELINE config 2, 3 or 5 (step roofline on the config's own
    algorithmic bytes; the phase / kernel breakdown comes from rocprofv3 of this command)."""
    import sys
    import torch
    sys.path.insert(0, ROOT)
    N, alg, work = CONFIGS[cfg]
    if cfg == 5:
        from pyrmt_amd.mac import MacMultiDisc
        sim = MacMultiDisc(N, n_discs=3, seed=3)
    elif cfg == 3:
        from pyrmt_amd.simulation import disc_in_taylor_green
        sim = disc_in_taylor_green(N, "weno5")
    else:
        from pyrmt_amd.simulation import soft_disc_in_lid_driven
        sim = soft_disc_in_lid_driven(N)
    sim.step(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sim.step(args.steps)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    d = sim.diagnostics()
    assert np.all(np.isfinite(np.asarray(d["cx"]))), "non-finite state"
    value = N * N * args.steps / el
    gbs = value * alg / 1e9
    out = {"metric": f"cell-updates/s (full RMT step) at N={N}; achieved HBM GB/s vs peak",
           "value": value, "unit": "cell-updates/s", "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": el / args.steps * 1e3, "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "f64",
           "data": "synthetic (the driver's own initial condition)",
           "config": {"workload": work, "grid": N, "baseline_config": cfg,
                      "parallelism": "single-gpu"},
           "roofline": {"bound": "hbm", "kernel": "whole step (every kernel of the loop body)",
                        "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                        "alg_bytes_per_cell": alg}}
    tf = PMC_TRAFFIC_CFG.get(cfg)
    if tf and os.path.exists(tf):
        # measured HBM bytes per step (FETCH x2 + WRITE passes of this command) and the rate
        # they imply at this line's step time
        tj = json.load(open(tf))
        per_step = tj["per_step"]["total"]
        out["roofline"].update({"traffic": per_step, "traffic_unit": "bytes per step",
                                "traffic_rev": tj.get("git_rev"),
                                "measured_GBs": per_step / (el / args.steps) / 1e9})
    if not args.no_cpu_baseline and cfg in (3, 5):
        out["cpu_baseline"] = cpu_baseline_cfg(cfg, N)
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4, choices=sorted(CONFIGS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--grid", "--n", dest="n", type=int, default=4096)
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if args.config != 4:
        if args.gpus != 1 or int(os.environ.get("WORLD_SIZE", "1")) != 1:
            raise SystemExit("--config 2/3/5: single-GPU lines (the multi-GPU line is config 4)")
        return main_config(args, args.config)

    ws, rank, local = _dist()
    import torch
    import torch.distributed as dist
    # RMT_DIST_BACKEND=gloo: rehearsal of the multi-rank path with every rank on the visible
    # GPUs round-robin (host-staged collectives); the default is RCCL, one rank per GPU
    backend = os.environ.get("RMT_DIST_BACKEND", "nccl")
    dev = local % torch.cuda.device_count() if backend == "gloo" else local
    torch.cuda.set_device(dev)
    # RMT_BENCH_DIST=1: the multi-rank path (process group, TorchComm slabs, barriers, MAX
    # over ranks) even at one rank -- the driver's N>1 code path rehearsed on one GPU
    md = ws > 1 or os.environ.get("RMT_BENCH_DIST") == "1"
    if md:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    import sys
    sys.path.insert(0, ROOT)
    N = args.n
    if md:
        from pyrmt_amd import distributed as D
        sim = D.soft_disc_in_lid_driven(N, D.TorchComm())
    else:
        from pyrmt_amd.simulation import soft_disc_in_lid_driven
        sim = soft_disc_in_lid_driven(N)
    sim.step(args.warmup)
    torch.cuda.synchronize()

    def timed(k):
        if md:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sim.step(k)
        torch.cuda.synchronize()
        if md:
            dist.barrier()
        el = time.perf_counter() - t0
        if md:
            t = torch.tensor([el], device="cuda", dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # `value`: the K steps with no profiling events; then the same K steps again with HIP
    # events around each phase and around the dominant kernel's launches (the roofline and
    # the phase breakdown come from this second timed region)
    elapsed = timed(args.steps)
    sim.set_profiling(True)
    elapsed_prof = timed(args.steps)
    ph = sim.phase_times()
    sim.set_profiling(False)
    d = sim.diagnostics()
    assert np.all(np.isfinite(d["cx"])) and np.all(np.isfinite(d["umax"])), "non-finite state"

    if rank == 0:
        cells = N * N * args.steps          # one problem (strong scaling when ws > 1)
        value = cells / elapsed
        traffic, step_traffic, pmc_rev = _pmc(N, 2 if md else 1)
        rk_ms, rk_intervals = ph["rk4_stage_kernels"]
        rk_launches = rk_intervals if not md else 4 * rk_intervals
        per_launch_s = rk_ms / 1e3 / rk_launches
        # achieved: SURVEY 8(d)'s algorithmic bytes of the stress + RK4 pass (7 planes per cell
        # for the 4 stage launches) spread over the launches, / the HIP-event launch time;
        # a slab's cell-updates are its owned rows (the recomputed halo rows are overhead)
        own = N * N if not md else (sim.slabs[0].r1 - sim.slabs[0].r0) * N
        alg_per_launch = RK4_ALG_BYTES_PER_CELL * own / 4
        achieved = alg_per_launch / per_launch_s / 1e9
        ex_ms, ex_calls = ph["extrap_sweep_kernel" if not md else "extrap_chain_kernel"]
        out = {
            "metric": "cell-updates/s (full RMT step) at N=4096; achieved HBM GB/s vs peak",
            "value": value, "unit": "cell-updates/s", "n_gpus": ws, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong",   # one N=4096 problem at every N
            "vs_baseline": None,
            "dtype": "f64", "data": "synthetic (driver initial condition: disc at rest, lid U=1)",
            "config": {"workload": f"soft_disc_in_lid_driven N={N} semilagrangian "
                                   "(configs 2/4 loop body)", "grid": N,
                       "parallelism": (f"slab{ws} (row slabs, {'RCCL' if backend == 'nccl' else backend})"
                                       if md else "single-gpu")},
            # the dominant HBM-bound kernel: the fused RK4 stage (4 launches per step)
            "roofline": {"bound": "hbm", "kernel": "k_mom_stage (fused RK4 stage, 4 launches/step)",
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_rev": pmc_rev,
                         "launch_ms": per_launch_s * 1e3,
                         "alg_bytes_per_launch": alg_per_launch},
            # ... whose own bound is the fp64 VALU issue rate (SQ counters)
            "compute_roofline": _f64_roof(N, 2 if md else 1, per_launch_s),
            # the dominant kernel by time is not HBM-bound: the exact raster-order extrapolation
            # chain runs on one workgroup, bounded by its dependency depth
            "latency_bound": {"kernel": "k_ex_chain (exact serial-order extrapolation chain)",
                              "ms_per_step": ex_ms / max(1, ex_calls),
                              "dag_depth_fits": _chain_depth(N),
                              "us_per_link": (ex_ms / max(1, ex_calls) * 1e3 / _chain_depth(N)
                                              if _chain_depth(N) else None),
                              "dag_source": "profiles/r05/chain_dag_n4096.json"},
            "step_roofline": {"alg_bytes_per_cell": STEP_ALG_BYTES_PER_CELL,
                              "per_gpu": True,
                              "achieved_GBs": value / ws * STEP_ALG_BYTES_PER_CELL / 1e9,
                              "frac": value / ws * STEP_ALG_BYTES_PER_CELL / 1e9 / HBM_PEAK_GBS,
                              "traffic_per_step": step_traffic,
                              "measured_GBs": (step_traffic / (elapsed / args.steps) / 1e9
                                               if step_traffic else None)},
            "ms_per_step_profiled": elapsed_prof / args.steps * 1e3,
            "phase_ms_per_step": {k: v[0] / max(1, args.steps) for k, v in ph.items()},
        }
        if not args.no_cpu_baseline and ws == 1:
            out["cpu_baseline"] = cpu_baseline(N, args.cpu_steps)
        print(json.dumps(out), flush=True)
    if md:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
