#!/usr/bin/env python3
"""Benchmark: multigrid V-cycles/s + level-1 smoother HBM GB/s vs roofline.

Workload (BASELINE.json configs[2], the 8192-element metric): the reference
mesh untitled8192.msh (128x32x2 triangles), n_split = 5 (8,388,608 fine
sub-elements, 25.2 M DOF; every level lives in HBM, well past the 256 MiB
Infinity Cache), multi_levels = 3, n_smooth = 4, solver = 3 (block
Gauss-Seidel), the reference's mode-9 physics (dt = 1.25e-5, k = 1,
omega = 0.8). One step = one V-cycle of transport_tri_semi.F90:319-379
(restriction leg, 15 coarse smoother calls, prolongation leg, halo after
every smoother call) over the whole mesh.

Defaults: the fused V-cycle (fused = 3) in its resident call schedule -- the K
cycles of a pamg_vcycle(K) call in ONE launch, every tile's state (all levels)
on-chip between cycles, loaded once and stored once (pamg_vcycle.hip k_vc_resb);
the state after the call is the per-step kernel sequence's, bit for bit (values
overwritten unread inside the call -- stores, and a smoother call's last sweep --
are not produced) -- and the
contracted operator arithmetic (arith = 1: fma rows of A_e = M/dt + Kd; ~1e-15
relative to the reference on the solution, the north star's bar being 1e-10).
The cycle is then fp64-issue-bound: the roofline is the fp64 operations the launch
executes (pamg_vcycle_flops x cycles) over its duration against the 78.6 TFLOP/s
fp64 peak. The other schedules (one HBM-bound launch per cycle: the round-1 form, with
its HBM roofline), the reference's own operation order (arith = 0, bitwise equal
to the reference) and the other workloads are timed and reported under "extra".

N > 1 (python -m torch.distributed.run ... bench.py --gpus N): strong scaling
of the same mesh, x-strip domain decomposition by unstructured element, one
process per GPU, halo words of remote neighbours packed by the level-1 launch
and exchanged with RCCL (grouped ncclSend/ncclRecv over xGMI) after the last
cycle of each pamg_vcycle call (every cycle rewrites every halo word and
nothing inside the call reads them; --halo-exchange 1 exchanges after every
cycle, overlapped with the next). `value` = V-cycles of the whole mesh / max
over ranks of the timed wall time.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time
from datetime import timedelta

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "p-a_multigrids_amd"))
MESH = os.path.join(ROOT, "tests", "meshes", "untitled8192.msh")
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# fp64 peak: MI355X spec FP64 vector 78.6 TFLOP/s (= the FP64 matrix peak; half the guide's 157.3
# TFLOP/s FP32 vector peak: a wave64 v_fma_f64 issues in 4 cycles per SIMD, 256 CUs x 4 SIMDs x 16
# lanes x 2 flops x 2.4 GHz)
FP64_PEAK_TFLOPS = 78.6
EVENT_STRIDE = 10
# the bound of every host collective of a multi-rank run (PAMG_BENCH_RENDEZVOUS_S overrides; tests use a short one)
RENDEZVOUS_S = int(os.environ.get("PAMG_BENCH_RENDEZVOUS_S", "300"))
ALL_CLASSES = 0x2FF7F   # every timing class (PAMG_K_*) but sweep_bench (bit 16 face_fallback counts regardless)
SWEEP_LAUNCHES = 60    # launches of each level-1 HBM sweep roofline measurement


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 warm-up cycles (~30 ms): after 5 (~1 ms) the GPU's clocks have not settled and the
    # timed region reads 6,550 instead of 7,460 V-cycles/s on the same box
    # (scripts/event_probe.py, archive/profiles/r01_v15_warmup.txt)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--nsplit", type=int, default=5)
    ap.add_argument("--levels", type=int, default=3)
    ap.add_argument("--nsmooth", type=int, default=4)
    ap.add_argument("--mesh", default=MESH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the n_split=3 and sweep-kernel side measurements")
    ap.add_argument("--extras-after", action="store_true",
                    help="run the side measurements after the timed region instead of before the warm-up")
    ap.add_argument("--halo-mode", type=int, default=0)
    ap.add_argument("--comm", choices=["rccl", "detached"], default="rccl",
                    help="detached: partitions without the RCCL exchange -- a check of the multi-process "
                         "orchestration on a one-GPU box (ranks share the GPU; timings are not a result)")
    ap.add_argument("--halo-exchange", type=int, default=0,
                    help="multi-rank: 0 exchange the level-1 halo once per pamg_vcycle call (after its last "
                         "cycle), 1 after every cycle")
    ap.add_argument("--arith", type=int, default=1,
                    help="1: contracted operator arithmetic (fma rows of A_e = M/dt + Kd; ~1e-15 of the reference, "
                         "the north star's bar is 1e-10); 0: the reference's operation order (bitwise)")
    ap.add_argument("--fused", type=int, default=3,
                    help="3: pipelined fused launches, level 1 of cycle c + coarse levels of cycle c+1 in one "
                         "launch (default); 1: two fused launches per V-cycle; 2: the same, concurrent on two "
                         "streams; 0: per-step kernels")
    return ap.parse_args()


def host_cpu():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def reference_proc(mesh_path, nsplit, ntime, nmg, core=0):
    """Start the reference's own fp64 build (oracle/_ref/pamg_ref_fp64) on a mesh, pinned to one core:
    (process, its scratch directory), or None without the build"""
    exe = os.path.join(ROOT, "oracle", "_ref", "pamg_ref_fp64")
    if not os.path.exists(exe):
        return None
    tmp = tempfile.mkdtemp(prefix="pamg_cpu_")
    shutil.copy(mesh_path, os.path.join(tmp, "mesh.msh"))
    with open(os.path.join(tmp, "pamg_ref.nml"), "w") as f:
        f.write(f"&pamg_ref\n pamg_mesh='mesh.msh', pamg_dump_prefix='', pamg_nsplit={nsplit}, "
                f"pamg_ntime={ntime},\n pamg_nmultigrid={nmg}, pamg_solver=3, pamg_levels=3, pamg_nsmooth=4, "
                f"pamg_vtk=100000\n/\n")
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = ["taskset", "-c", str(core), exe] if shutil.which("taskset") else [exe]
    return subprocess.Popen(cmd, cwd=tmp, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, env=env), tmp


def reference_wait(pt, timeout=900):
    """the seconds of a reference run's `cpu_time for time_loop` window (transport_tri_semi.F90:297-387),
    or None"""
    if pt is None:
        return None
    p, tmp = pt
    try:
        out, _ = p.communicate(timeout=timeout)
        m = re.search(r"cpu_time for time_loop =\s*([0-9.Ee+-]+)", out)
        return float(m.group(1)) if p.returncode == 0 and m else None
    except subprocess.TimeoutExpired:
        p.kill()
        p.communicate()
        return None
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def run_reference(mesh_path, nsplit, ntime, nmg, timeout=900):
    """The reference's own fp64 build (1 core) on a mesh: its time_loop window in seconds, or None"""
    return reference_wait(reference_proc(mesh_path, nsplit, ntime, nmg), timeout)


CPU_STRIP = (32, 8)   # 512 un_eles: 1/16 of untitled8192's, the same 4**5 sub-elements each
CPU_SHARE = 16        # host cores of a one-GPU share of the box (OMP_NUM_THREADS there)


CPU_PAIRS = 3        # independent (1-cycle, 3-cycle) run pairs of the 1-core baseline; the median is reported


def spaced_cores(n):
    """n cores of this process's affinity set, spread out (distinct core complexes where there are many)"""
    cores = sorted(os.sched_getaffinity(0))
    if len(cores) <= n:
        return cores[:n]
    step = len(cores) // n
    return [cores[i * step] for i in range(n)]


def cpu_baseline():
    """Reference CPU path on this host, measured at the benchmarked n_split = 5 and L = 3: the
    reference Fortran itself (fp64 build, oracle/_ref, 1 core, its own `cpu_time for time_loop`
    window) on a bounded sample -- one time step of 1 and of 3 V-cycles on a 512-element
    synthetic strip; half the difference is the steady-state cost of one V-cycle (the first cycle
    of a run carries a one-off cost the others do not, and it varies from run to run: round 5's
    single 2-minus-1 difference read 5.5 s on one box and 9.1 s on another). CPU_PAIRS pairs run at
    once, each process pinned to its own core (spread over the core complexes); the median pair is
    the value and the spread is reported. The reference's work is per un_ele (stencils re-derived per
    un_ele visit, then its 4**n_split sub-elements; nothing couples un_eles in mode 9), so
    untitled8192's 8192 un_eles take 16x as long; the 16x is checked against the full-size run by
    scripts/cpu_baseline_probe.py (profiles/r05_final_cpu_baseline_probe.txt: 150.05 s per V-cycle)."""
    import pamg
    tmp = tempfile.mkdtemp(prefix="pamg_cpu_msh_")
    try:
        path = os.path.join(tmp, "strip.msh")
        strip = pamg.Mesh.strip(*CPU_STRIP)
        strip.write_msh(path)
        U = strip.U
        cores1 = spaced_cores(2 * CPU_PAIRS)
        procs = [reference_proc(path, 5, 1, nmg, cores1[2 * i + (nmg == 3)]) for i in range(CPU_PAIRS) for nmg in (1, 3)]
        ts = [reference_wait(p) for p in procs]
        pairs = [(ts[2 * i], ts[2 * i + 1]) for i in range(CPU_PAIRS)]
        diffs = sorted((b - a) / 2 for a, b in pairs if a is not None and b is not None and b > a)
        t1 = sorted(a for a, _ in pairs if a is not None)
        t1 = t1[len(t1) // 2] if t1 else None
        # the same sample on every core of the GPU's host share at once: the reference is serial and its mode-9
        # un_eles are uncoupled, so CPU_SHARE strips (1/16 of the mesh each) run as independent processes, one
        # per core -- the all-cores figure beside the 1-core baseline
        ncores = max(1, min(CPU_SHARE, len(os.sched_getaffinity(0))))
        cores = sorted(os.sched_getaffinity(0))[:ncores]
        tall = {}
        for nmg in (1, 2):
            procs = [reference_proc(path, 5, 1, nmg, c) for c in cores]
            tall[nmg] = [reference_wait(p) for p in procs]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    if not diffs:
        return None
    scale = 8192 / U
    tc = diffs[len(diffs) // 2]
    allc = None
    if all(v is not None for v in tall[1] + tall[2]):
        steady = sorted(b - a for a, b in zip(tall[1], tall[2]))
        tcn = steady[len(steady) // 2]
        allc = dict(value=ncores / (scale * tcn), unit="V-cycles/s", cores=ncores,
                    sample=f"{ncores} copies of the same strip sample at once, one per core (the reference is serial; "
                           f"mode 9's un_eles are uncoupled, so partitions are independent runs): median steady-state "
                           f"V-cycle {tcn:.2f} s per strip (1 core alone: {tc:.2f} s); value = {ncores} / "
                           f"({scale:g} x {tcn:.2f} s)")
    return dict(value=1.0 / (scale * tc), unit="V-cycles/s", cores=1, kind="reference", all_cores=allc,
                sample=f"reference fp64 build (flang -O2) on 1 core of '{host_cpu()}' at n_split=5, multi_levels=3, "
                       f"n_smooth=4 on a {U}-element synthetic strip ({CPU_STRIP[0]}x{CPU_STRIP[1]}x2): {CPU_PAIRS} pairs of "
                       f"one time step of 1 and of 3 V-cycles (each process on its own core), steady-state V-cycle = "
                       f"(t3 - t1) / 2 per pair = {', '.join(f'{d:.2f}' for d in diffs)} s, median {tc:.2f} s; value = "
                       f"1 / ({scale:g} x {tc:.2f} s), scaled to untitled8192's 8192 elements (the reference's work is "
                       f"linear in the element count; full-size check 150.05 s per V-cycle, "
                       f"profiles/r05_final_cpu_baseline_probe.txt)",
                pair_seconds=[[round(a, 2) if a else None, round(b, 2) if b else None] for a, b in pairs],
                steady_cycle_s=[round(d, 3) for d in diffs],
                spread=round(diffs[-1] / diffs[0], 3) if diffs[0] > 0 else None,
                seconds_1cycle=t1, host_cpu=host_cpu())


SKIP_DIGEST = ("pamg_face.hip", "pamg_mesh.cpp", "pamg_vtu.cpp")


def source_digest():
    """sha256 over the kernel sources (p-a_multigrids_amd/csrc, include/pamg.h): a committed PMC
    summary applies to the build it was measured on only (scripts/pmc_summary.py records it)."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "p-a_multigrids_amd", "csrc")
    # every source the op = 0 kernels and their launch path are built from: all of csrc but the face
    # operator's kernels (pamg_face.hip), the mesh reader and the VTU writer, which none of them uses
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")) and f not in SKIP_DIGEST)
    for f in files + ["../../include/pamg.h"]:
        h.update(f.encode())
        h.update(open(os.path.join(csrc, f), "rb").read())
    return h.hexdigest()[:16]


def pmc_traffic(kernel, nsplit, levels, info=None):
    """HBM bytes per launch of the roofline kernel from the committed rocprofv3
    PMC summary (profiles/pmc_<kernel>.json), if one exists for this config and was
    measured on these kernel sources (else None: a stale file is not reported)."""
    p = os.path.join(ROOT, "profiles", f"pmc_{kernel.lower()}.json")
    try:
        d = json.load(open(p))
        if int(d.get("n_split", -1)) == nsplit and int(d.get("levels", levels)) == levels:
            match = d.get("source_digest") == source_digest()
            if info is not None:
                info.update({"file": os.path.relpath(p, ROOT), "commit": d.get("commit"),
                             "source_digest": d.get("source_digest"), "source_matches_build": match})
            return d.get("hbm_bytes_per_launch") if match else None
    except Exception:
        pass
    return None


RK_DESC = {"vcycle_res": "k_vc_resb (resident V-cycle call: all cycles of the call in one launch, every level of a "
                         "tile on-chip between cycles; fp64-issue-bound)",
           "vcycle_pipe": "k_vc_fine<.., true> (pipelined fused V-cycle: level 1 of cycle c -- both smoother "
                          "calls, residual, restrictor, prolongator -- and levels 2..L of cycle c+1, per tile)",
           "vcycle": "k_vc_fine (fused V-cycle, level-1 launch: both smoother calls, residual, prolongator; "
                     "the coarse levels run in k_vc_coarse just before it)",
           "smooth_L1": "k_smooth (level-1 smoother call, n_smooth sweeps fused)"}


TIME_LOOP_STEPS = 50


def measure_time_loop(s):
    """The time loop as the reference drives it (transport_tri_semi.F90:299-381): pamg_run of
    TIME_LOOP_STEPS steps, each begin_timestep (told := tnew, level-1 RHS) + n_multigrid = 2
    V-cycles. Wall time without events; then the same loop with an event pair around every
    launch for the per-launch algorithmic bytes, the kernel time and the roofline of the
    launch that starts each step (told, RHS and the step's constant halo words)."""
    s.timing_enable(0)
    s.run(10, 2)   # warm-up
    s.synchronize()
    t0 = time.perf_counter()
    s.run(TIME_LOOP_STEPS, 2)
    s.synchronize()
    el = time.perf_counter() - t0
    s.timing_enable(ALL_CLASSES)
    s.timing_stride(1)
    s.timing_reset()
    s.run(TIME_LOOP_STEPS, 2)
    s.synchronize()
    tm = s.timing()
    s.timing_enable(0)
    by = sum(v["bytes"] / v["launches"] * v["issued"] for v in tm.values() if v["launches"]) / TIME_LOOP_STEPS
    kms = sum(v["ms"] for v in tm.values() if v["launches"]) / TIME_LOOP_STEPS
    ms_step = 1e3 * el / TIME_LOOP_STEPS
    fl = 2 * s.vcycle_flops()
    # a step moves the state in and out once (HBM) and runs 2 cycles of fp64 work: both rooflines
    out = {"workload": f"pamg_run(ntime={TIME_LOOP_STEPS}, n_multigrid=2): each step begin_timestep + 2 V-cycles "
                       "(the reference's n_multigrid loop inside its time loop); with the resident schedule the whole run is "
                       "one launch",
           "vcycles_per_s": round(2 * TIME_LOOP_STEPS / el, 1), "ms_per_step": round(ms_step, 4),
           "alg_bytes_per_step": by, "achieved": round(by / (ms_step * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": round(by / (ms_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "fp64_flops_per_step": fl, "fp64_tflops": round(fl / (ms_step * 1e-3) / 1e12, 2),
           "fp64_frac": round(fl / (ms_step * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
           "kernel_ms_per_step_evented": round(kms, 4),
           "launches": {k: dict(per_step=round(v["issued"] / TIME_LOOP_STEPS, 2),
                                ms=round(v["ms"] / v["launches"], 4),
                                alg_bytes=v["bytes"] / v["launches"],
                                frac=round(v["bytes"] / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4))
                        for k, v in tm.items() if v["launches"]}}
    return out


def measure_workload(pamg, m, S, L, ns, arith, device, cycles=100):
    """V-cycles/s of one pamg_vcycle(cycles) call on mesh m at n_split S (after a warm-up call),
    and its launch's fp64 roofline from an evented pass"""
    s = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=3, device=device, arith=arith, fused=3)
    s.begin_timestep()
    s.vcycle(cycles)
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(cycles)
    s.synchronize()
    v = cycles / (time.perf_counter() - t0)
    s.timing_enable(ALL_CLASSES)
    s.timing_stride(EVENT_STRIDE)
    s.timing_reset()
    s.vcycle(cycles)
    s.synchronize()
    tm = s.timing()
    out = dict(U=m.U, n_split=S, fine_sub_elements=m.U * 4 ** S, vcycles_per_s=round(v, 1))
    k = tm["vcycle_res"]
    if k["launches"]:
        ms = k["ms"] / k["launches"]
        fl = s.vcycle_flops() * cycles
        out.update(launch_ms=round(ms, 4), fp64_tflops=round(fl / (ms * 1e-3) / 1e12, 2),
                   fp64_frac=round(fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4))
    s.close()
    return out


def measure_face(pamg, m, S, L, device, cycles=20, cycle=0):
    """the face-coupled operator (op = 1) on mesh m: V-cycles/s of the reference's
    cycle (cycle = 0) or the corrected one (cycle = 1; n_smooth 4, red-black GS) and, from an evented
    pass, each kernel class's time and algorithmic bytes per cycle; the level-1 sweeps (HBM-bound)
    against the HBM roofline"""
    s = pamg.SemiImplicitIterative(m, S, L, n_smooth=4, solver=3, device=device, op=1, cycle=cycle)
    s.begin_timestep()
    s.vcycle(3)
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(cycles)
    s.synchronize()
    dt = (time.perf_counter() - t0) / cycles
    s.timing_enable(ALL_CLASSES)
    s.timing_stride(1)
    s.timing_reset()
    s.vcycle(cycles)
    s.synchronize()
    tm = s.timing()
    out = dict(n_split=S, levels=L, n_smooth=4, vcycles_per_s=round(1 / dt, 1), ms_per_cycle=round(dt * 1e3, 4),
               kernels={k: dict(launches_per_cycle=v["launches"] // cycles, ms_per_cycle=round(v["ms"] / cycles, 4),
                                gbs=round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None)
                        for k, v in tm.items() if v["launches"]})
    k1 = tm["smooth_L1"]
    if k1["launches"] and k1["ms"] > 0:
        # level 1's launches: one sweep each, or two (k_face_pp, the default); a cycle executes 2 (n_smooth - 1)
        # level-1 sweeps (a smoother call's last sweep only in the call's last cycle), the
        # corrected cycle 2 n_smooth
        gbs = k1["bytes"] / (k1["ms"] * 1e-3) / 1e9
        lpc = k1["launches"] / cycles
        spl = (2 * 4 if cycle else 2 * (4 - 1)) / lpc
        out["roofline_level1_launch"] = dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                                             frac=round(gbs / HBM_PEAK_GBS, 4), sweeps_per_launch=round(spl, 2),
                                             ms_per_launch=round(k1["ms"] / k1["launches"], 4),
                                             ms_per_sweep=round(k1["ms"] / k1["launches"] / spl, 4))
    s.close()
    return out


def measure_corrected(pamg, m, S, L, ns, arith, device, cycles=200):
    """the corrected V-cycle (cycle = 1: the fresh residual restricted, coarse
    levels from zero, the interpolated coarse correction added) on the benchmarked workload. A
    pamg_vcycle call runs as one resident launch (k_vc_corr, every level of a tile on-chip between the
    cycles; bitwise the per-step sequence, tests/test_corrected.py): V-cycles/s of a `cycles`-cycle
    call after a warm-up call, the launch's fp64 roofline from an evented pass, and the per-step
    kernel sequence beside it (fused = 0, 20 cycles)"""
    s = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=3, device=device, arith=arith, cycle=1)
    s.begin_timestep()
    s.vcycle(cycles)
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(cycles)
    s.synchronize()
    v = cycles / (time.perf_counter() - t0)
    s.timing_enable(1 << 14)   # PAMG_K_VCYCLE_CORR
    s.timing_stride(1)
    s.timing_reset()
    s.vcycle(cycles)
    s.synchronize()
    k = s.timing()["vcycle_corr"]
    out = dict(workload=f"corrected V-cycle (cycle=1), n_split={S} L={L} n_smooth={ns} GS, one pamg_vcycle({cycles}) "
                        "call = one resident launch", vcycles_per_s=round(v, 1))
    if k["launches"]:
        ms = k["ms"] / k["launches"]
        fl = s.vcycle_flops() * cycles
        out.update(launch_ms=round(ms, 4), fp64_flops_per_cycle=s.vcycle_flops(),
                   fp64_tflops=round(fl / (ms * 1e-3) / 1e12, 2),
                   fp64_frac=round(fl / (ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4))
    s.close()
    s0 = pamg.SemiImplicitIterative(m, S, L, n_smooth=ns, solver=3, device=device, arith=arith, cycle=1, fused=0)
    s0.begin_timestep()
    s0.vcycle(3)
    s0.synchronize()
    t0 = time.perf_counter()
    s0.vcycle(20)
    s0.synchronize()
    out["per_step_vcycles_per_s"] = round(20 / (time.perf_counter() - t0), 1)
    s0.close()
    return out


def comm_report(s, world, dist):
    kind, ver, path = s.comm_info()
    mine = {"transport": kind, "rccl_version": ver, "librccl": path}
    if world == 1:
        return [mine]
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return allr


def main():
    a = parse()
    time_loop = None
    roofline_hbm = None
    extra_pre = {}
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            raise SystemExit("--gpus N > 1 must be launched with torch.distributed.run (one process per GPU)")
    # torch first: libpamg then binds the same HIP / RCCL runtime (shared sonames)
    import torch
    import torch.distributed as dist
    import pamg

    if world > 1:
        # every host collective is bounded (RENDEZVOUS_S): a rank that never joins, or never reaches the
        # communicator's creation, ends the run with an error line instead of a hang -- RCCL's own initialisation
        # cannot be bounded (pamg_comm_init, profiles/r06_rccl_init_probe.txt), so every rank meets here first
        dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=RENDEZVOUS_S))
    mesh = pamg.Mesh.read(a.mesh)

    def comm_for(_mode=None):
        if world == 1:
            return None
        if a.comm == "detached":   # orchestration check on one GPU: no RCCL, no exchange
            return (world, rank, None, mesh.x_strip_owner(world))
        obj = [pamg.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        dist.barrier()   # all ranks hold the id and enter pamg_comm_init together
        return (world, rank, obj[0], mesh.x_strip_owner(world))

    comm = comm_for()
    ndev = max(1, torch.cuda.device_count())
    device = local % ndev
    if torch.cuda.is_available():
        torch.cuda.set_device(device)   # torch's own synchronize() then stays on this rank's GPU
    s = pamg.SemiImplicitIterative(mesh, a.nsplit, a.levels, n_smooth=a.nsmooth, solver=3, device=device,
                                   halo_mode=a.halo_mode, comm=comm, fused=a.fused, arith=a.arith,
                                   halo_exchange=a.halo_exchange)
    s.begin_timestep()
    if rank == 0 and world == 1 and not a.no_extra:
        # the north star's HBM roofline: one level-1 sweep of the assembled element-block-sparse
        # operator, 168 B per sub-element (x, b, out, the 3x3 block, omega/D), and the matrix-free sweep beside
        # it; HIP events around SWEEP_LAUNCHES launches each (tests/test_roofline_kernels.py pins their output).
        # Measured first, on the same handle (the sweeps write a scratch buffer only), so the V-cycle's warm-up and
        # timed call follow ~30 ms of GPU work (profiles/r05_a_shape_probe.txt: +2 % over an idle GPU's first call)
        for asm in (False, True):
            ms, by = s.sweep_bench(SWEEP_LAUNCHES, asm)
            extra_pre["sweep_assembled" if asm else "sweep_stencil"] = dict(
                ms=round(ms, 4), bytes_per_launch=by, gbs=round(by / (ms * 1e-3) / 1e9, 1),
                frac=round(by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3), launches=SWEEP_LAUNCHES)
            if asm:
                roofline_hbm = {"bound": "hbm", "kernel": "k_sweep_assembled (one level-1 Jacobi sweep over the "
                                "assembled block-CSR operator, matrices.F90:997-1198; contracted arithmetic)",
                                "achieved": round(by / (ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                "traffic": pmc_traffic("sweep_assembled", a.nsplit, 1),
                                "alg_bytes_per_launch": by, "bytes_per_sub_element": 168,
                                "sub_elements": mesh.U * 4 ** a.nsplit, "ms_per_launch": round(ms, 4),
                                "events": f"HIP event pair around each of {SWEEP_LAUNCHES} launches"}
    def other_measurements():
        """the side measurements reported under "extra" (and time_loop); the time loop last, on the bench's
        own handle, so that with the default order the warm-up and the timed call follow it without an idle gap"""
        nonlocal time_loop
        ex = {}
        # the round-1 form on the same workload: one HBM-bound launch per cycle (call schedule 1),
        # its pipelined launch against the HBM roofline
        s1 = pamg.SemiImplicitIterative(mesh, a.nsplit, a.levels, n_smooth=a.nsmooth, solver=3, device=device,
                                        fused=a.fused, arith=a.arith)
        s1.set_call_schedule(1)
        s1.begin_timestep()
        s1.vcycle(a.warmup)
        s1.synchronize()
        t0 = time.perf_counter()
        s1.vcycle(a.steps)
        s1.synchronize()
        v1 = a.steps / (time.perf_counter() - t0)
        s1.timing_enable(ALL_CLASSES)
        s1.timing_stride(EVENT_STRIDE)
        s1.timing_reset()
        s1.vcycle(a.steps)
        s1.synchronize()
        kp = s1.timing()["vcycle_pipe"]
        if kp["launches"]:
            msp = kp["ms"] / kp["launches"]
            bp = kp["bytes"] / kp["launches"]
            ex["one_launch_per_cycle"] = dict(
                vcycles_per_s=round(v1, 1), pipe_ms=round(msp, 4), pipe_alg_bytes=bp,
                pipe_gbs=round(bp / (msp * 1e-3) / 1e9, 1), pipe_frac=round(bp / (msp * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                pipe_traffic=pmc_traffic("vcycle_pipe", a.nsplit, a.levels))
        s1.close()
        # the matrices.F90 SpMV (csr_mul_array, 3 entries per row) over the level-1 operator's
        # size in the reference's block numbering: 3 N1 rows, 52 B per row (3 x (4 B column +
        # 8 B value), 8 B result, 8 B of the gathered vector)
        nrows = 3 * mesh.U * 4 ** a.nsplit
        base = 3 * (np.arange(nrows, dtype=np.int32) // 3)
        jloc = (base[:, None] + np.arange(1, 4, dtype=np.int32)[None, :]).reshape(-1)
        del base
        sp = pamg.Sparse(s, np.arange(1, 3 * nrows, 3, dtype=np.int32), jloc,
                         np.random.default_rng(20251015).uniform(-1, 1, 3 * nrows))
        del jloc
        ms = sp.bench(nrows, 20)
        by = 52.0 * nrows
        ex["csr_mul_array"] = dict(rows=nrows, ms=round(ms, 4), bytes_per_launch=by,
                                   gbs=round(by / (ms * 1e-3) / 1e9, 1),
                                   frac=round(by / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3))
        sp.close()
        # the same workload in the other schedules / arithmetic: the per-step kernel sequence
        # (bitwise equal to the fused cycle), the concurrent fused launches, and the reference's
        # operation order (bitwise equal to the reference)
        for tag, kw in (("fused0", dict(fused=0, arith=a.arith)), ("fused1", dict(fused=1, arith=a.arith)),
                        ("fused2", dict(fused=2, arith=a.arith)), ("fused3", dict(fused=3, arith=a.arith)),
                        ("arith0", dict(fused=a.fused, arith=0)), ("arith1", dict(fused=a.fused, arith=1))):
            if kw["fused"] == a.fused and kw["arith"] == a.arith:
                continue
            su = pamg.SemiImplicitIterative(mesh, a.nsplit, a.levels, n_smooth=a.nsmooth, solver=3, device=device,
                                            **kw)
            su.begin_timestep()
            su.vcycle(a.warmup)
            su.synchronize()
            t0 = time.perf_counter()
            su.vcycle(a.steps)
            su.synchronize()
            ex[f"{tag}_vcycles_per_s"] = round(a.steps / (time.perf_counter() - t0), 2)
            su.close()
        s3 = pamg.SemiImplicitIterative(mesh, 3, a.levels, n_smooth=a.nsmooth, solver=3, device=device,
                                        arith=a.arith)
        s3.begin_timestep()
        s3.vcycle(a.warmup)
        s3.synchronize()
        t0 = time.perf_counter()
        s3.vcycle(max(a.steps, 200))
        s3.synchronize()
        ex["nsplit3_vcycles_per_s"] = round(max(a.steps, 200) / (time.perf_counter() - t0), 1)
        # config 3 driven as the reference drives it: pamg_run(50, 2), one resident launch
        s3.run(5, 2)
        s3.synchronize()
        t0 = time.perf_counter()
        s3.run(TIME_LOOP_STEPS, 2)
        s3.synchronize()
        ex["nsplit3_time_loop_vcycles_per_s"] = round(2 * TIME_LOOP_STEPS / (time.perf_counter() - t0), 1)
        s3.close()
        # the other workloads of the north star on one GPU: config 5's mesh at n_split = 6 (tiles are
        # quarters of an un_ele there), config 3 at n_split = 6, and a synthetic structured strip
        # 4x untitled8192 (256 x 64 x 2, pamg_msh_strip) at the benchmarked n_split = 5
        for tag, m_, S_ in (("irregular_nsplit6", pamg.Mesh.read(os.path.join(ROOT, "tests", "meshes", "irregular.msh")), 6),
                            ("untitled8192_nsplit6", mesh, 6),
                            ("strip256x64_nsplit5", pamg.Mesh.strip(256, 64), 5)):
            ex[tag] = measure_workload(pamg, m_, S_, a.levels, a.nsmooth, a.arith, device)
        # the face-coupled operator on the benchmarked mesh, n_split 5, 3 levels
        ex["op1"] = measure_face(pamg, mesh, a.nsplit, 3, device)
        # and the corrected cycle on it (cycle = 1: levels 1-2 in two-sweep passes, the coarsest level's chain)
        ex["op1_cycle1"] = measure_face(pamg, mesh, a.nsplit, 3, device, cycle=1)
        ex["cycle1"] = measure_corrected(pamg, mesh, a.nsplit, a.levels, a.nsmooth, a.arith, device)
        time_loop = measure_time_loop(s)
        return ex

    extra_other = {}
    if rank == 0 and world == 1 and not a.no_extra and not a.extras_after:
        # before the warm-up (default): the timed call then starts on a GPU that has been running this
        # workload for a while, its clocks settled, as in a deployment's steady state, instead of on a GPU
        # coming out of the idle host work around handle creation (profiles/r05_p_extras_order.txt)
        extra_other = other_measurements()
    s.vcycle(a.warmup)
    s.synchronize()
    # per-kernel HIP events (the roofline) inside the timed region on one GPU; with N ranks
    # each rank's share of a cycle is ~1/N as long and the events would be a visible part of
    # it, so there they are recorded in a short pass after the timed region
    live_events = world == 1
    s.timing_enable(ALL_CLASSES if live_events else 0)
    # an event pair between back-to-back launches costs ~10 us (~5 % of a cycle): time the
    # first launch of each class and then one in EVENT_STRIDE
    s.timing_stride(EVENT_STRIDE)
    s.timing_reset()

    def barrier():
        if world > 1:
            dist.barrier()

    # Timed region: one barrier aligns the ranks' starts; then each rank times its own call from
    # its own synchronized stream (no host collective inside the timed region: a gloo barrier is
    # tens to hundreds of us of TCP, a large part of a rank's 20-cycle call at N = 8) and the
    # elapsed times are reduced with MAX afterwards. The barrier's own cost is measured beside it.
    barrier_us = None
    if world > 1:
        bt = []
        for _ in range(5):
            t0 = time.perf_counter()
            dist.barrier()
            bt.append(time.perf_counter() - t0)
        barrier_us = 1e6 * float(np.median(bt))
    barrier()
    torch.cuda.synchronize()
    s.synchronize()
    t0 = time.perf_counter()
    s.vcycle(a.steps)
    s.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    rank_elapsed = [elapsed]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        rank_elapsed = [None] * world
        dist.all_gather_object(rank_elapsed, t1 - t0)
        barrier()
    if not live_events:
        # per-launch events time each launch on its own: the post-pass runs the pipelined
        # calls as one launch per cycle (the timed region ran the partition's automatic
        # schedule, two tile streams)
        post = max(1, min(a.steps, 20))
        resident = a.fused == 3 and a.halo_exchange == 0 and a.levels >= 2
        if not resident:
            s.set_call_schedule(1)
        s.timing_enable(ALL_CLASSES)
        s.timing_reset()
        s.vcycle(post)
        s.synchronize()
    tm = s.timing()
    value = a.steps / elapsed
    # dominant kernel by total time inside the timed region
    dom = max((k for k in tm if tm[k]["launches"] > 0 and k != "sweep_bench"), key=lambda k: tm[k]["ms"])
    # roofline kernel: the resident call when it ran (fp64-bound), else the fused V-cycle's
    # pipelined launch or the level-1 smoother (HBM-bound)
    rk = next(k for k in ("vcycle_res", "vcycle_pipe", "vcycle", "smooth_L1") if tm[k]["launches"])
    kinfo = tm[rk]
    ms_per_launch = kinfo["ms"] / max(1, kinfo["launches"])
    bytes_per_launch = kinfo["bytes"] / max(1, kinfo["launches"])
    achieved = bytes_per_launch / (ms_per_launch * 1e-3) / 1e9 if ms_per_launch > 0 else 0.0
    traffic_src = {}
    traffic = pmc_traffic(rk, a.nsplit, a.levels, traffic_src) if world == 1 else None
    cycles_per_launch = (a.steps if live_events else post) if rk == "vcycle_res" else 1
    flops_per_launch = s.vcycle_flops() * cycles_per_launch
    tflops = flops_per_launch / (ms_per_launch * 1e-3) / 1e12 if ms_per_launch > 0 else 0.0
    extra = {"kernels": {k: dict(ms_total=round(v["ms"], 4), launches=v["launches"], issued=v["issued"],
                                 gbs=round(v["bytes"] / (v["ms"] * 1e-3) / 1e9, 1) if v["ms"] > 0 else None)
                         for k, v in tm.items() if v["launches"]},
             "dominant_kernel": dom, "fine_sub_elements_per_rank": s.U * 4 ** a.nsplit}
    # whole-cycle algorithmic bytes over the whole-cycle time (every launch of the timed region:
    # bytes per sampled launch x launches issued)
    tot_bytes = sum(v["bytes"] / v["launches"] * v["issued"] for v in tm.values() if v["launches"])
    extra["cycle_alg_bytes"] = tot_bytes / a.steps
    extra["cycle_alg_gbs"] = round(tot_bytes / elapsed / 1e9, 1)
    extra["comm"] = comm_report(s, world, dist)
    if world > 1:
        extra["rank_ms_per_step"] = [round(1e3 * v / a.steps, 5) for v in rank_elapsed]
        extra["barrier_us"] = round(barrier_us, 1)
        # each rank's resident kernel per cycle (post-pass events), beside the timed ms_per_step
        kk = [None] * world
        dist.all_gather_object(kk, ms_per_launch / cycles_per_launch)
        extra["rank_kernel_ms_per_cycle"] = [round(v, 5) for v in kk]
        # the per-call exchange started early (post-pass call): per rank (exchange start, exchange end,
        # resident launch end) in us from the launch's start -- end < launch end: hidden behind the launch
        xt = s.early_exchange_times() if not live_events else None
        xa = [None] * world
        dist.all_gather_object(xa, [round(v, 1) for v in xt] if xt else None)
        extra["early_exchange_us"] = xa
    if rank == 0 and world == 1 and not a.no_extra and a.extras_after:
        extra_other = other_measurements()
    if rank == 0 and world == 1 and not a.no_extra:
        extra.update(extra_pre)
        extra.update(extra_other)
    if world > 1 and not a.no_extra:
        # the other exchange mode on the same partition (timed region the same shape): halo words
        # exchanged after every cycle, overlapped with the next one
        mode = 1 - a.halo_exchange
        sx = pamg.SemiImplicitIterative(mesh, a.nsplit, a.levels, n_smooth=a.nsmooth, solver=3, device=device,
                                        halo_mode=a.halo_mode, comm=comm_for(mode), fused=a.fused, arith=a.arith,
                                        halo_exchange=mode)
        sx.begin_timestep()
        sx.vcycle(a.warmup)
        sx.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sx.vcycle(a.steps)
        sx.synchronize()
        t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        extra[f"halo_exchange{mode}_vcycles_per_s"] = round(a.steps / float(t.item()), 2)
        extra[f"halo_exchange{a.halo_exchange}_vcycles_per_s"] = round(value, 2)
        sx.close()
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline()
        if cpu:
            extra["speedup_vs_cpu"] = round(value / cpu["value"], 1)
            if time_loop:
                extra["time_loop_speedup_vs_cpu"] = round(time_loop["vcycles_per_s"] / cpu["value"], 1)
    if rank == 0:
        line = {
            "metric": "multigrid V-cycles/sec + smoother HBM GB/s vs roofline, 8192-ele tri mesh",
            "value": round(value, 3),
            "unit": "V-cycles/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * elapsed / a.steps, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "reference mesh untitled8192.msh, deterministic mode-9 IC/source (no random data)",
            "config": {"workload": f"untitled8192.msh n_split={a.nsplit} multi_levels={a.levels} "
                                   f"n_smooth={a.nsmooth} GS; a step = one V-cycle over the whole mesh, the "
                                   f"{a.steps} timed steps issued as one pamg_vcycle({a.steps}) call inside one time "
                                   f"step (the reference-shaped loop, 2 V-cycles per time step: time_loop)",
                       "fine_sub_elements": mesh.U * 4 ** a.nsplit, "levels": a.levels,
                       "parallelism": f"dd{world}", "halo_mode": a.halo_mode,
                       "arith": "contracted (fma, 1e-15 of the reference)" if a.arith else "reference order (bitwise)",
                       "fused": a.fused, "halo_exchange": "per call" if a.halo_exchange == 0 else "per cycle",
                       "comm": a.comm if world > 1 else None,
                       "call_schedule": ("resident (the call's cycles in one launch)" if rk == "vcycle_res" else
                                         "two tile streams" if world > 1 else "one launch per cycle")},
            "roofline": ({"bound": "fp64-valu", "kernel": RK_DESC[rk],
                          "events": (f"timed region (the call is one launch)" if live_events
                                     else f"post-pass of one call of {post} cycles"),
                          "achieved": round(tflops, 2), "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(tflops / FP64_PEAK_TFLOPS, 4), "traffic": traffic,
                          "traffic_source": traffic_src or None,
                          "fp64_flops_per_launch": flops_per_launch, "cycles_per_launch": cycles_per_launch,
                          "alg_bytes_per_launch": bytes_per_launch, "hbm_gbs": round(achieved, 1),
                          "ms_per_launch": round(ms_per_launch, 4)}
                         if rk == "vcycle_res" else
                         {"bound": "hbm", "kernel": RK_DESC[rk],
                          "events": (f"timed region, the first and then 1 in {EVENT_STRIDE} launches" if live_events
                                     else "post-pass of min(steps, 20) cycles, one launch per cycle"),
                          "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                          "alg_bytes_per_launch": bytes_per_launch, "ms_per_launch": round(ms_per_launch, 4)}),
            "roofline_hbm_smoother": roofline_hbm,
            "cpu_baseline": ({k: cpu[k] for k in ("value", "unit", "cores", "kind", "sample", "all_cores")} if cpu else None),
            "time_loop": time_loop,
            "extra": extra,
        }
        print(json.dumps(line), flush=True)
    s.close()
    if world > 1:
        dist.destroy_process_group()


def error_line(e):
    """one JSON line naming the failing rank and the error (the run exits non-zero)"""
    return json.dumps({"metric": "multigrid V-cycles/sec + smoother HBM GB/s vs roofline, 8192-ele tri mesh",
                       "value": None, "error": f"{type(e).__name__}: {e}", "rank": int(os.environ.get("RANK", "0")),
                       "world_size": int(os.environ.get("WORLD_SIZE", "1"))})


if __name__ == "__main__":
    try:
        main()
    except SystemExit:
        raise
    except BaseException as e:  # noqa: BLE001 -- reported as the run's JSON line, then a non-zero exit
        print(error_line(e), flush=True)
        sys.exit(1)
