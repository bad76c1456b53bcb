#!/usr/bin/env python3
"""Benchmark of the MI355X encoder hot path (BASELINE.json metric: encoder audio-frames/s on 30 s clips).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config {q4k64,f16x1,f16x64,q80x64,q80bf16x64}]

A "step" = one pass of the hot path (PCM -> log-mel -> conv -> 32 blocks -> pool+LN) over one batch of
synthetic 30 s / 16 kHz clips per GPU, PCM already resident in HBM when the timed region starts.
Default workload = BASELINE.json configs[2] ("batch=64 30 s clips, Q4_K quantized weights, 1xMI355X"); at N
GPUs every rank runs its own 64 clips (weak scaling; N=8 is configs[3], batch=512 sharded 64/GPU). Weights are
synthetic (deterministic splitmix64 generator at the real Qwen2-Audio encoder shapes), generated and quantized
on rank 0, packed into the device layout and broadcast to every rank with one RCCL broadcast.

Prints ONE JSON line on rank 0. Multi-GPU: `python bench.py --gpus N` launches N ranks itself (torchrun as a child
process, started before this process touches any GPU); the driver's own `torchrun --nproc-per-node N bench.py --gpus N`
works the same way. A WORLD_SIZE that disagrees with --gpus is an error, never a silent 1-GPU run.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd")
sys.path.insert(0, PKG)

CONFIGS = {
    # name: (ggml weight type, clips per GPU, BASELINE.json config it reproduces)
    "q4k64": ("q4_k", 64, "configs[2]: batch=64 30 s clips, Q4_K quantized weights, 1xMI355X per rank"),
    "f16x1": ("f16", 1, "configs[1]: single 30 s synthetic 16 kHz clip, fp16 weights, 1xMI355X per rank"),
    "f16x64": ("f16", 64, "batch=64 30 s clips, fp16 weights (F16 path at the configs[2] batch)"),
    "q4kx1": ("q4_k", 1, "single 30 s synthetic 16 kHz clip, Q4_K weights (the configs[2] contract at batch 1)"),
    "q80x64": ("q8_0", 64, "batch=64 30 s clips, Q8_0 weights (exact Q8_0 x Q8_0 contract)"),
    # configs[4] per rank: Q8_0 file, weights dequantized to bf16, bf16 inter-op activations (Q2A_ACT_BF16)
    "q80bf16x64": ("q8_0", 64, "configs[4] per rank: batch=64 30 s clips (512 over 8 GPUs), Q8_0 weights + bf16 "
                               "activations (Q2A_ACT_BF16: bf16-dequantized weights, bf16 MFMA, fp32 accumulation)"),
}
T_MEL = 3000              # mel frames per 30 s clip (10 ms hop) -> the metric's "audio frame"
N_SAMPLES = 480000
# algorithmic work per clip: 2 273.77 GFLOP; weight GEMMs 1 887.44; attention 368.64; conv 17.69
D, F, T, L = 1280, 5120, 1500, 32
FLOP_FC1_PER_CLIP = 2.0 * T * F * D
FLOP_WEIGHT_GEMMS_PER_CLIP = 2.0 * T * (3 * D * D + D * D + F * D + D * F) * L
FLOP_PER_CLIP = FLOP_WEIGHT_GEMMS_PER_CLIP + 2 * 2.0 * T * T * D * L + 2.0 * (2 * T) * D * 384 + 2.0 * T * D * 3 * D
PEAK_FP16_MFMA_TFLOPS = 2500.0    # MI355X dense fp16/bf16 MFMA (MI355X_MICROARCH.md, chip table)
PROF_NAMES = ["mel", "conv1", "conv2", "layernorm", "gemm_qkv", "attention", "quant_act", "gemm_o", "gemm_fc1",
              "gemm_fc2", "pool_ln"]


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def make_model(wt: str, workdir: str, threads: int) -> str:
    import q2a
    base = os.path.join(workdir, "full-f16.bin")
    if not os.path.exists(base):
        subprocess.check_call([q2a.TOOL_PATH, "gen-model", base, "full", "f16", "0x51A2", str(threads)])
    if wt == "f16":
        return base
    path = os.path.join(workdir, f"full-{wt}.bin")
    if not os.path.exists(path):
        subprocess.check_call([q2a.TOOL_PATH, "quantize", base, path, wt, str(threads)])
    return path


def synth_clips(first: int, n: int) -> np.ndarray:
    host = C.CDLL(os.path.join(PKG, "lib", "libq2a_host.so"))
    out = np.empty((n, N_SAMPLES), dtype=np.float32)
    for i in range(n):
        host.q2a_synth_clip(C.c_void_p(out[i].ctypes.data), C.c_int64(N_SAMPLES), C.c_int(first + i))
    return out


# the reference CPU builds (oracle/Makefile): x86-64-v3 (AVX2 / FMA / F16C, runs on any host) and x86-64-v4 (AVX-512:
# the ggml kernels a GGML_NATIVE build picks on the GPU box's EPYC 9575F)
REF_BUILDS = {"x86-64-v3": "_ref", "x86-64-v4 (avx512)": "_ref_avx512"}


def _ref_encode(model_path: str, clip: str, workdir: str, threads: int, reps: int, build: str = "_ref") -> dict | None:
    harness = os.path.join(ROOT, "oracle", build, "ref_harness")
    if not os.path.exists(harness):
        return None
    outp = os.path.join(workdir, "ref_out.f32")
    try:
        r = subprocess.run([harness, "encode", model_path, clip, outp, str(threads), str(reps)], check=True,
                           capture_output=True, text=True, timeout=600)
    except Exception as ex:  # noqa: BLE001
        log("cpu baseline failed:", ex)
        return None
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_baseline(model_path: str, wt: str, workdir: str, reps: int) -> dict | None:
    """The reference ggml CPU path itself (oracle/_ref*/ref_harness: /root/reference's sources compiled -O3 at
    -march=x86-64-v3 AND -march=x86-64-v4 (AVX-512, what a GGML_NATIVE build picks on this box), kind "reference"; the
    faster build is the headline, both in legs.isa) timed on this box's host cores, one synthetic 30 s clip per rep through
    whisper_full, clips run sequentially on one context. Legs (~25 s of CPU work in all):
      main     the workload's weight type, n_threads = the CPU share this process may use (affinity, capped by
               OMP_NUM_THREADS: the box allots 16 host CPUs per GPU; lscpu / nproc are recorded beside it)
      default  same weights, n_threads = min(4, hw) — examples/main/main.cpp:33's default
      f16x1    configs[1] (fp16 weights, one clip) at the main thread count (when the workload is not F16)
      whole_box the workload's weights at n_threads = the box's PHYSICAL cores (lscpu sockets x cores per socket), one
               clip — the box-level CPU figure (what the 8 GPUs of the box share); its affinity / cgroup limits are
               recorded in `host`, since a process confined to fewer CPUs than threads time-slices them."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_ref", "ref_harness")):
        return None
    hw = host_cpu_info()
    share = hw["affinity"] or 1
    if hw["omp_num_threads"] and hw["omp_num_threads"].isdigit():
        share = min(share, int(hw["omp_num_threads"]))
    clip = os.path.join(workdir, "clip0.f32")
    synth_clips(0, 1)[0].tofile(clip)
    # the main leg on every reference build present; the FASTER one is the headline (its ISA named in `sample`)
    isa_runs = {}
    for isa, build in REF_BUILDS.items():
        r = _ref_encode(model_path, clip, workdir, share, reps, build)
        if r is not None:
            isa_runs[isa] = (build, r)
    if not isa_runs:
        return None
    isa = min(isa_runs, key=lambda k: isa_runs[k][1]["mean_s"])
    best, main = isa_runs[isa]
    legs = {"isa": {k: {"value": round(T_MEL / r["mean_s"], 2), "s_per_clip": round(r["mean_s"], 3), "threads": share,
                        "weights": wt} for k, (_, r) in isa_runs.items()}}
    dflt_threads = min(4, hw["os_cpu_count"] or 4)
    d = _ref_encode(model_path, clip, workdir, dflt_threads, 1, best)
    if d:
        legs["default_threads"] = {"value": round(T_MEL / d["mean_s"], 2), "threads": dflt_threads, "weights": wt,
                                   "s_per_clip": round(d["mean_s"], 3)}
    phys = _physical_cores(hw)
    if phys and phys > share:
        wb = _ref_encode(model_path, clip, workdir, phys, 1, best)
        if wb:
            legs["whole_box"] = {"value": round(T_MEL / wb["mean_s"], 2), "threads": phys, "weights": wt,
                                 "s_per_clip": round(wb["mean_s"], 3), "affinity_cpus": hw.get("affinity"),
                                 "cgroup_cpu_max": hw.get("cgroup_cpu_max")}
    if wt != "f16":
        f16 = _ref_encode(os.path.join(workdir, "full-f16.bin"), clip, workdir, share, 1, best)
        if f16:
            legs["configs1_f16x1"] = {"value": round(T_MEL / f16["mean_s"], 2), "threads": share, "weights": "f16",
                                      "s_per_clip": round(f16["mean_s"], 3)}
    return {"value": round(T_MEL / main["mean_s"], 2), "unit": "audio-frames/s", "cores": share,
            "kind": "reference",
            "sample": f"{reps} x one 30 s clip ({wt} weights) through whisper_full (ggml CPU backend, n_threads={share}, "
                      f"-O3 -march={isa.split()[0]}: the faster of the builds in legs.isa), mean {main['mean_s']:.2f} s/clip",
            "isa": isa,
            "gflops_per_s": round(FLOP_PER_CLIP / main["mean_s"] / 1e9, 1),
            "legs": legs, "host": hw}


def _physical_cores(hw: dict) -> int | None:
    try:
        return int(hw["lscpu_sockets"]) * int(hw["lscpu_cores_per_socket"])
    except (KeyError, ValueError):
        return None


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`--gpus N` without a torchrun environment: run this script as N ranks (one process per GPU) under
    torch.distributed.run as a CHILD process and return its exit code. Called before anything initialises the GPU
    (only device_count, which does not, on this image): the parent never holds a GPU context."""
    import torch
    have = torch.cuda.device_count()
    if have < n and os.environ.get("Q2A_BENCH_REHEARSE") != "1":
        log(f"bench: --gpus {n} but only {have} visible device(s)")
        return 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def host_cpu_info() -> dict:
    """What the CPU baseline ran on: the box's CPUs (nproc / lscpu) and the share this process may use."""
    info = {"os_cpu_count": os.cpu_count()}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except AttributeError:
        info["affinity"] = os.cpu_count()
    info["omp_num_threads"] = os.environ.get("OMP_NUM_THREADS")
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            info["cgroup_cpu_max"] = f.read().strip()
    except OSError:
        pass
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        want = ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core", "CPU(s)")
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in want:
                info["lscpu_" + k.strip().replace("(s)", "s").replace(" ", "_").lower()] = v.strip()
    except Exception:  # noqa: BLE001
        pass
    return info


# The profile set measured on the current tree; its summaries are cited ahead of older rounds' (tags do not sort
# by date: r04y was taken after r04z, and r05w, not r05x, is the round-5 closing set). Round 6: r06ad, the closing set
# after the late-round load fixes (r06o before them).
PROFILE_TAG = "r06ad"


def _profile_files(names) -> list:
    """Committed summaries, oldest first by tag, the PROFILE_TAG set last (the one the line cites)."""
    return sorted(names, key=lambda f: (f.startswith(PROFILE_TAG + "_"), f))


def fc1_kernel_label(wt: str, bf16: bool, M: int) -> str:
    """The k_gemm instantiation the engine launches for fc1 (N = 5120, K = 1280), mirroring q2a_gemm.hip's tile
    regimes: 256x256 8-phase tiles once ceil(M/256) x 20 tiles >= 512 (M >= 6401), persistent (PIPE 2) for the Q4_K
    pre-activation at whole 256-row tiles, else 128x128 two-stage tiles."""
    epi = "GELU_H" if (bf16 or wt != "q4_k") else "PRE_H"
    blk = "BF16" if bf16 else {"q4_k": "256", "f16": "0", "q8_0": "32"}[wt]
    if (M + 255) // 256 * 20 >= 512 and blk != "32":
        pipe = 2 if (epi == "PRE_H" and M % 256 == 0) else 1
        return f"k_gemm<256,256,2,4,{epi},{blk},{pipe}>"
    if (M + 255) // 256 * 20 >= 512:
        return f"k_gemm<128,256,2,4,{epi},{blk},0>"
    return f"k_gemm<128,128,2,2,{epi},{blk},0>"


# the matrix-core kernel classes (Q2A_PROF_*: QKV, attention, O, fc1, fc2), one launch per layer each
ROOF_CLASSES = (4, 5, 7, 8, 9)


def roof_flop_per_launch(cls: int, clips: int) -> float:
    """Algorithmic flops of one launch of a class: 2.M.N.K for the weight GEMMs (M = 1500 x clips),
    4.T^2.D per clip for the attention (QK^T and P.V)."""
    M = T * clips
    return {4: 2.0 * M * 3 * D * D, 5: 2 * 2.0 * T * T * D * clips, 7: 2.0 * M * D * D, 8: 2.0 * M * F * D,
            9: 2.0 * M * D * F}[cls]


def roof_label(cls: int, wt: str, bf16: bool, clips: int) -> str:
    M = T * clips
    if cls == 5:
        return ("attention (k_attn_pp<true>: bf16 contract, one bf16 MFMA per product)" if bf16 else
                "attention (k_attn_t: F32-class contract, 3 fp16 MFMA terms per product), T=1500 D=1280 H=20")
    if cls == 8:
        return "gemm_fc1 (%s), M=%d N=5120 K=1280" % (fc1_kernel_label(wt, bf16, M), M)
    return {4: "gemm_qkv, M=%d N=3840 K=1280", 7: "gemm_o, M=%d N=1280 K=1280",
            9: "gemm_fc2 (8-phase main rounds + 128x128 tail at 64 clips), M=%d N=1280 K=5120"}[cls] % M


def committed_counter(config: str, cls: int, suffix: str, field: str):
    """A kernel class's figure from the committed profile summaries of this workload (the PROFILE_TAG set last)."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None, None
    files = _profile_files(f for f in os.listdir(pdir) if f.endswith(f"_{config}_{suffix}.json"))
    if not files:
        return None, None
    with open(os.path.join(pdir, files[-1])) as f:
        kern = json.load(f)["kernels"]
    name = PROF_NAMES[cls]
    for k, e in kern.items():
        if (k == name or e.get("class") == name) and field in e:
            return e[field], "profiles/" + files[-1]
    return None, None


def mfma_util_of(config: str, clips: int):
    """The metric's "MFMA util %" over a whole step, from the committed PROFILE_TAG profile set of this workload: every
    kernel's SQ MFMA-busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over its active cycles,
    profiles/sq_summary.py) weighted by its rocprofv3 time per step, over the step time measured under rocprofv3 by the
    same collection. Kernels without MFMA work count as 0. None when the set lacks any of the three summaries."""
    if clips != CONFIGS[config][1]:
        return None
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for tag in (PROFILE_TAG,):   # (an older set's kernel names need not match the current tree's)
        sq_f, st_f, b_f = (f"{tag}_{config}_sq_mfma.json", f"{tag}_{config}_rocprof_kernel_stats.csv",
                           f"{tag}_{config}_bench_under_rocprof.json")
        if not all(os.path.exists(os.path.join(pdir, f)) for f in (sq_f, st_f, b_f)):
            continue
        import csv
        with open(os.path.join(pdir, sq_f)) as f:
            # keys "class | kernel name" (profiles/sq_summary.py)
            busy = {k.split(" | ", 1)[-1]: e["mfma_busy_frac"] for k, e in json.load(f)["kernels"].items()
                    if "mfma_busy_frac" in e}
        with open(os.path.join(pdir, b_f)) as f:
            b = json.loads(f.read().strip().splitlines()[-1])
        with open(os.path.join(pdir, st_f)) as f:
            rows = list(csv.DictReader(f))
        # steps in the traced run (warm-up, timed, breakdown and dominant-class passes): one attention launch per layer
        steps = sum(int(r["Calls"]) for r in rows if "k_attn" in r["Name"]) / 32
        if steps <= 0:
            continue
        weighted = sum(busy.get(r["Name"], 0.0) * float(r["TotalDurationNs"]) for r in rows) / steps / 1e6
        return {"value": round(weighted / b["ms_per_step"], 4), "mfma_busy_ms_per_step": round(weighted, 2),
                "step_ms_under_rocprof": b["ms_per_step"],
                "sources": [f"profiles/{sq_f}", f"profiles/{st_f}", f"profiles/{b_f}"],
                "definition": "sum over kernels of SQ MFMA-busy fraction x rocprofv3 time per step, over the step time"}
    return None


def roofline_of(cls: int, timed_ms, timed_n, config: str, wt: str, bf16: bool, clips: int) -> dict:
    """roofline object of one class: achieved = algorithmic flops per launch / its average launch time (HIP events on
    the engine's stream over the timed region), against the dense fp16 / bf16 MFMA peak (the MFMA dtype issued, also
    for the integer k-quant dots); traffic = HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE, separate passes)
    and the SQ MFMA busy fraction from the committed summaries of this workload."""
    avg_s = timed_ms[cls] / max(1, timed_n[cls]) / 1e3
    flop = roof_flop_per_launch(cls, clips)
    achieved = flop / avg_s / 1e12 if avg_s > 0 else 0.0
    same_batch = clips == CONFIGS[config][1]
    traffic, tsrc = committed_counter(config, cls, "pmc_traffic", "hbm_bytes_per_launch_corrected") if same_batch else (None, None)
    busy, bsrc = committed_counter(config, cls, "sq_mfma", "mfma_busy_frac") if same_batch else (None, None)
    r = {"bound": "mfma", "kernel": roof_label(cls, wt, bf16, clips), "achieved": round(achieved, 1),
         "peak": PEAK_FP16_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP16_MFMA_TFLOPS, 4),
         "traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": tsrc,
         "flop_per_launch": flop, "avg_launch_ms": round(avg_s * 1e3, 4), "launches_timed": int(timed_n[cls]),
         "mfma_busy_frac": round(busy, 4) if busy is not None else None, "mfma_busy_source": bsrc}
    if cls == 5 and not bf16:
        r.update({"issued_tflops": round(3 * achieved, 1), "issued_frac": round(3 * achieved / PEAK_FP16_MFMA_TFLOPS, 4),
                  "issued_note": "3 fp16 MFMA terms per algorithmic product (F32-class QK^T and P.V, DESIGN.md §2)"})
    return r


def c_group_leg(args, model_path: str, clips_per_gpu: int) -> dict:
    """The one-process multi-GPU C ABI (q2a_group_open_with + q2a_group_encode_host) at the visible
    device count, in a child process (this one holds its own engine; the child's failure or hang cannot take the
    bench line with it): an engine from the model file, ONE RCCL broadcast of its device-layout weights to every other
    visible device, then clips_per_gpu x devices clips from pageable host memory (PCIe both ways included)."""
    cmd = [sys.executable, os.path.abspath(__file__), "--c-group-child", "--config", args.config, "--workdir",
           args.workdir, "--clips", str(clips_per_gpu)]
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=dict(os.environ, Q2A_GROUP_MODEL=model_path))
        if r.returncode != 0:
            return {"error": f"rc {r.returncode}: " + r.stderr.strip()[-300:]}
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception as ex:  # noqa: BLE001
        return {"error": str(ex)[:300]}


def c_group_child(args) -> None:
    import q2a
    model_path = os.environ["Q2A_GROUP_MODEL"]
    t0 = time.time()
    eng = q2a.Engine(model_path, device=0, act=q2a.ACT_BF16 if "bf16" in args.config else q2a.ACT_REFERENCE)
    t_open = time.time() - t0
    t0 = time.time()
    g = q2a.Group(engine=eng)
    t_group = time.time() - t0
    n = g.size * args.clips
    pcm = synth_clips(0, n)
    clips = [pcm[c] for c in range(n)]
    out = np.empty((n,) + g.out_shape, dtype=np.float32)
    g.encode_host(clips, out=out)   # staging buffers and workspaces grown here
    reps = 2
    ts = time.perf_counter()
    for _ in range(reps):
        _, st = g.encode_host(clips, out=out)
    dt = (time.perf_counter() - ts) / reps
    assert (st == q2a.CLIP_ENCODED).all() and np.isfinite(out).all()
    res = {"devices": g.size, "clips": n, "frames_per_s": round(n * T_MEL / dt, 1), "s_per_call": round(dt, 4),
           "engine_open_s": round(t_open, 3), "group_open_s": round(t_group, 3), "setup": g.setup_times(),
           "source": "q2a_group_open_with over an engine opened from the model file; q2a_group_encode_host from "
                     "pageable host arrays (PCIe in and out included), one host thread per device"}
    g.close()
    eng.close()
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="q4k64", choices=sorted(CONFIGS))
    ap.add_argument("--clips", type=int, default=0, help="override clips per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-legs", action="store_true",
                    help="skip the PCIe-inclusive and host-API legs (profiles/collect.sh: every launch is then the workload's own batch)")
    ap.add_argument("--cpu-reps", type=int, default=2)   # ~7 s of reference CPU work on 16 threads (+ legs)
    ap.add_argument("--workdir", default=os.environ.get("Q2A_BENCH_DIR", os.path.join(tempfile.gettempdir(), "q2a_bench")))
    ap.add_argument("--no-c-group", action="store_true", help="skip the one-process multi-GPU C ABI leg (c_group)")
    ap.add_argument("--c-group-child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.c_group_child:
        return c_group_child(args)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    ws, rank, local = dist_env()
    if ws != args.gpus:
        log(f"bench: WORLD_SIZE={ws} but --gpus {args.gpus}: refusing to report a mislabelled run")
        sys.exit(2)
    import torch
    # Q2A_BENCH_REHEARSE=1: rehearse the N>1 path on a 1-GPU box (every rank on device 0, gloo collectives on host
    # tensors); the numbers of such a run are not a scaling measurement
    rehearse = os.environ.get("Q2A_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    torch.cuda.set_device(local)
    coll_dev = "cpu" if rehearse else "cuda"
    dist = None
    # Q2A_BENCH_PG=1: bring up the process group (RCCL) at world size 1 too, so a 1-GPU box executes the N>1 path's
    # collectives (communicator init on the device, the blob broadcast, the max-over-ranks all-reduce, barriers)
    if ws > 1 or os.environ.get("Q2A_BENCH_PG") == "1":
        import torch.distributed as dist
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    import q2a
    from q2a import dist as qd

    wt, clips_per_gpu, workload = CONFIGS[args.config]
    if args.clips:
        clips_per_gpu = args.clips
    threads = min(16, os.cpu_count() or 8)
    os.makedirs(args.workdir, exist_ok=True)

    # ---- model: rank 0 generates + quantizes + packs; one RCCL broadcast of the packed blob over xGMI
    t0 = time.time()
    model_path = None
    blob_host = None
    if rank == 0:
        model_path = make_model(wt, args.workdir, threads)
        # the compact transport form (ggml weight rows: Q4_K at 144 B per 256 weights); each rank expands it into the
        # device layout on its own GPU when it opens the engine
        blob_host = q2a.pack_model(model_path, q2a.ACT_BF16 if "bf16" in args.config else q2a.ACT_REFERENCE, compact=True)
    t_bcast = 0.0
    if dist is not None:
        dist.barrier()
    tb = time.time()
    blob = qd.broadcast_blob(dist, blob_host, rank, coll_dev).cuda()
    torch.cuda.synchronize()
    if dist is not None:
        t_bcast = time.time() - tb
    del blob_host
    nbytes = blob.numel()
    tx = time.time()
    eng = q2a.Engine(device=local, device_blob=blob.data_ptr(), blob_size=nbytes)   # expands on the GPU (owns it)
    t_expand = time.time() - tx
    del blob
    eng.reserve(clips_per_gpu)
    t_setup = time.time() - t0

    # ---- inputs resident in HBM before the timed region (each rank its own clips)
    shard = qd.clip_range(rank, ws, clips_per_gpu)
    pcm = torch.from_numpy(synth_clips(shard.start, len(shard))).cuda()
    out = torch.empty((clips_per_gpu,) + eng.out_shape, dtype=torch.float32, device="cuda")
    ns = [N_SAMPLES] * clips_per_gpu

    def step():
        eng.encode_device(pcm.data_ptr(), N_SAMPLES, ns, out.data_ptr())

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    lib = q2a.lib()
    lib.q2a_profile_enable_mask.argtypes = [C.c_void_p, C.c_uint]
    prof_ms = (C.c_double * 11)()
    prof_n = (C.c_int64 * 11)()
    # the dominant matrix-core class (QKV, attention, O, fc1, fc2 = Q2A_PROF_* 4, 5, 7, 8, 9) from one profiled step
    # before the timed region; inside the timed region HIP events bracket only that class's launches (on the stream
    # the kernels run on). An event pair costs ~9 us of GPU time per launch (profiles/r06e_vrows_persistent_qkv_ab.json:
    # 128 pairs = 1.1 ms per step at one clip), under 0.2 % of a step from 8 clips up; below that the same events run
    # over an identical pass right after the timed region instead, so `value` carries none. The per-kernel breakdown of
    # every class comes from a separate fully-profiled pass.
    lib.q2a_profile_enable_mask(C.c_void_p(eng.h), sum(1 << i for i in ROOF_CLASSES))
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 1)
    step()
    torch.cuda.synchronize()
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 1)
    dominant = max(ROOF_CLASSES, key=lambda i: prof_ms[i])
    events_in_timed = clips_per_gpu >= 8
    lib.q2a_profile_enable_mask(C.c_void_p(eng.h), (1 << dominant) if events_in_timed else 0)
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 1)

    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    if not events_in_timed:   # the dominant class's events over an identical pass (small batches)
        lib.q2a_profile_enable_mask(C.c_void_p(eng.h), 1 << dominant)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 0)
    timed_ms, timed_n = list(prof_ms), list(prof_n)
    # breakdown pass (not timed): every kernel class bracketed by events
    brk_steps = max(1, min(args.steps, 3))
    lib.q2a_profile_enable(C.c_void_p(eng.h), 1)
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 1)
    for _ in range(brk_steps):
        step()
    torch.cuda.synchronize()
    lib.q2a_profile_read(C.c_void_p(eng.h), prof_ms, prof_n, 11, 0)
    lib.q2a_profile_enable(C.c_void_p(eng.h), 0)
    if not os.environ.get("Q2A_DIAG_BUILD"):   # diagnostic A/B libraries (diag/) compute garbage on purpose
        assert torch.isfinite(out).all().item(), "non-finite encoder output"

    elapsed = qd.max_over_ranks(dist, elapsed, coll_dev)

    # PCIe-inclusive rate (outside `value`): a serving loop over consecutive batches from pinned host memory, double
    # buffered — batch i+1's PCM goes host -> HBM and batch i-1's embd_enc HBM -> host on a copy stream while batch i
    # encodes (events order each buffer's reuse); the first upload and the last download are exposed
    pcie_steps = 0 if args.no_host_legs else 4
    pcm_host = pcm.cpu().pin_memory()
    out_host = [torch.empty(out.shape, dtype=out.dtype).pin_memory() for _ in range(2)]
    pcm_d, out_d = [pcm, torch.empty_like(pcm)], [out, torch.empty_like(out)]
    comp, cps = torch.cuda.current_stream(), torch.cuda.Stream()
    ev = {k: [torch.cuda.Event(), torch.cuda.Event()] for k in ("h2d", "comp", "d2h")}
    torch.cuda.synchronize()
    tp = time.perf_counter()
    for i in range(pcie_steps):
        b = i & 1
        with torch.cuda.stream(cps):
            if i >= 2:
                cps.wait_event(ev["comp"][b])
            pcm_d[b].copy_(pcm_host, non_blocking=True)
            ev["h2d"][b].record(cps)
        comp.wait_event(ev["h2d"][b])
        if i >= 2:
            comp.wait_event(ev["d2h"][b])
        eng.encode_device(pcm_d[b].data_ptr(), N_SAMPLES, ns, out_d[b].data_ptr(), stream=comp.cuda_stream)
        ev["comp"][b].record(comp)
        with torch.cuda.stream(cps):
            cps.wait_event(ev["comp"][b])
            out_host[b].copy_(out_d[b], non_blocking=True)
            ev["d2h"][b].record(cps)
    torch.cuda.synchronize()
    pcie_rate = qd.max_over_ranks(dist, time.perf_counter() - tp, coll_dev)
    pcie_rate = pcie_steps * clips_per_gpu * ws * T_MEL / pcie_rate if pcie_steps else None
    del pcm_d, out_d
    # the C host API itself (q2a_encode_host: pageable caller arrays, chunked + double-buffered inside), one call
    host_rate = None
    if clips_per_gpu >= 2 and not args.no_host_legs:
        pcm_np = [pcm_host[c].numpy() for c in range(clips_per_gpu)]
        out_np = np.empty((clips_per_gpu,) + eng.out_shape, dtype=np.float32)
        eng.encode_host(pcm_np, out=out_np)   # staging buffers allocated (and the output pages touched) here
        th = time.perf_counter()
        eng.encode_host(pcm_np, out=out_np)
        host_rate = qd.max_over_ranks(dist, time.perf_counter() - th, coll_dev)
        host_rate = clips_per_gpu * ws * T_MEL / host_rate
    total_clips = clips_per_gpu * ws * args.steps
    value = total_clips * T_MEL / elapsed

    if rank != 0:
        eng.close()
        if dist is not None:
            dist.destroy_process_group()
        return

    per_kernel = {PROF_NAMES[i]: {"ms_per_step": round(prof_ms[i] / brk_steps, 3),
                                  "launches_per_step": int(prof_n[i] // brk_steps)} for i in range(11)}
    gemm_ms = prof_ms[4] + prof_ms[7] + prof_ms[8] + prof_ms[9]
    gemm_tf = FLOP_WEIGHT_GEMMS_PER_CLIP * clips_per_gpu * brk_steps / (gemm_ms / 1e3) / 1e12
    bf16 = "bf16" in args.config
    # every matrix-core kernel class against the same fp16 MFMA peak, ALGORITHMIC flops: the
    # attention's F32-class contract issues 3 MFMA terms per product and the conv's exact accumulation 3 operand
    # parts, neither counted here
    for i, fl in ((1, 2.0 * (2 * T) * D * 3 * 128), (2, 2.0 * T * D * 3 * D), (4, 2.0 * T * 3 * D * D * L),
                  (5, 2 * 2.0 * T * T * D * L), (7, 2.0 * T * D * D * L), (8, FLOP_FC1_PER_CLIP * L), (9, 2.0 * T * D * F * L)):
        if prof_ms[i] > 0:
            tf = fl * clips_per_gpu * brk_steps / (prof_ms[i] / 1e3) / 1e12
            per_kernel[PROF_NAMES[i]].update({"tflops": round(tf, 1), "mfma_frac": round(tf / PEAK_FP16_MFMA_TFLOPS, 4)})
            if i == 5 and not bf16:
                # the MFMA work the reference contract's attention issues: S = Kh.Qh + Kl.Qh + Kh.Ql and
                # O += Vh.Ph + Vh.Pl + Vl.Ph, three 16x16x32 products per algorithmic one
                per_kernel[PROF_NAMES[i]].update({"issued_tflops": round(3 * tf, 1),
                                                  "issued_mfma_frac": round(3 * tf / PEAK_FP16_MFMA_TFLOPS, 4)})

    # the roofline objects: the DOMINANT kernel class (largest time per step among the matrix-core classes, each one
    # launch per layer; its events over the timed region) and the fc1 GEMM (north_star's "Q4_K encoder matmuls"; its
    # events of the breakdown pass unless it is the dominant class)
    roofline = roofline_of(dominant, timed_ms, timed_n, args.config, wt, bf16, clips_per_gpu)
    roofline["dominant"] = True
    roofline["avg_launch_source"] = ("HIP events on the launch stream over the timed region" if events_in_timed else
                                     "HIP events on the launch stream over an identical pass after the timed region "
                                     "(events cost ~9 us per launch, 5 % of a one-clip step)")
    roofline["share_of_step"] = round(prof_ms[dominant] / brk_steps / (elapsed / args.steps * 1e3), 4)
    if dominant == 8:
        roofline_fc1 = dict(roofline)
    else:
        roofline_fc1 = roofline_of(8, list(prof_ms), list(prof_n), args.config, wt, bf16, clips_per_gpu)
        roofline_fc1["avg_launch_source"] = "HIP events of the breakdown pass"
    roofline_fc1.pop("dominant", None)
    roofline_fc1["all_weight_gemms_tflops"] = round(gemm_tf, 1)

    cpu = None
    if ws == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(model_path, wt, args.workdir, args.cpu_reps)
    c_group = None
    if ws == 1 and not args.no_c_group and not args.no_host_legs:
        c_group = c_group_leg(args, model_path, clips_per_gpu)

    res = {
        "metric": "encoder audio-frames/sec (30 s clips) at 1/2/4/8 MI355X; MFMA util %",
        "value": round(value, 1),
        "unit": "audio-frames/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16 MFMA (fp32 acc), q8_0 weights dequantized to bf16, bf16 activations" if "bf16" in args.config else
                 {"q4_k": "q4_k x q8_k integer dots on fp16 MFMA (fp32 acc)", "f16": "fp16 MFMA (fp32 acc)",
                  "q8_0": "q8_0 x q8_0 integer dots on fp16 MFMA (fp32 acc)"}[wt],
        "data": "synthetic (deterministic 30 s / 16 kHz clips; random-init weights at Qwen2-Audio encoder shapes)",
        "config": {"workload": workload, "model": "qwen2-audio-encoder L32 D1280 H20 F5120 (synthetic weights)",
                   "weights": wt, "clips_per_gpu": clips_per_gpu, "global_batch": clips_per_gpu * ws,
                   "seq_len": T_MEL, "parallelism": f"dp{ws}"},
        "clips_per_s": round(total_clips / elapsed, 3),
        "tflops_total": round(FLOP_PER_CLIP * total_clips / elapsed / 1e12, 1),
        "roofline": roofline,
        "roofline_gemm_fc1": roofline_fc1,
        "mfma_util": mfma_util_of(args.config, clips_per_gpu),
        "cpu_baseline": cpu,
        "c_group": c_group,
        "pcie_inclusive_frames_per_s": round(pcie_rate, 1) if pcie_rate else None,
        "pcie_inclusive_source": f"{pcie_steps} batches from pinned host memory, H2D / D2H double-buffered on a copy stream",
        "host_api_frames_per_s": round(host_rate, 1) if host_rate else None,
        "per_kernel": per_kernel,
        "per_kernel_source": f"separate pass of {brk_steps} step(s), every kernel class bracketed by HIP events",
        "setup_s": {"total": round(t_setup, 1), "weight_h2d_plus_rccl_broadcast": round(t_bcast, 4), "weight_blob_bytes": nbytes, "weight_device_bytes": int(eng.info.weight_bytes),
                    "weight_expand_on_gpu": round(t_expand, 4),
                    "collective_backend": dist.get_backend() if dist is not None else None},
    }
    print(json.dumps(res), flush=True)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
