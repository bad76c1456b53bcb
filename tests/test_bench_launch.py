"""The multi-GPU launch glue of bench.py: `--gpus N` starts N ranks under torch.distributed.run
as a child process, a WORLD_SIZE that disagrees with --gpus exits 2 instead of reporting a mislabelled run, and a
2-rank run returns ONE JSON line labelled n_gpus 2 / dp2. The RCCL path itself needs an 8-GPU node (the driver's
SCALE run); on a 1-GPU box the 2 ranks are rehearsed on device 0 with gloo collectives (Q2A_BENCH_REHEARSE=1)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "Q2A_BENCH_REHEARSE")}
    e.update(kw)
    return e


def test_world_size_mismatch_exits_2():
    """A torchrun environment of 2 ranks with --gpus 1: refused before any GPU work (CPU-only check)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--no-cpu-baseline"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "WORLD_SIZE=2 but --gpus 1" in r.stderr
    assert r.stdout.strip() == ""


def test_more_gpus_than_visible_exits_2():
    """--gpus 2 on a host without 2 visible devices (and no rehearsal): exit 2, no ranks started."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("host has >= 2 GPUs")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--no-cpu-baseline"], capture_output=True, text=True,
                       timeout=120, env=_env())
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "only" in r.stderr and "visible" in r.stderr


@pytest.mark.gpu
def test_bench_two_ranks_rehearsal(tmp_path):
    """`python bench.py --gpus 2` (2 ranks, every rank on device 0, gloo) -> one JSON line, n_gpus 2, dp2, weak
    scaling over the 2 x 2 clips, setup timing of the blob broadcast present."""
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", "2", "--steps", "2", "--warmup", "1", "--clips", "2",
                        "--config", "f16x1", "--no-cpu-baseline", "--workdir", str(tmp_path)],
                       capture_output=True, text=True, timeout=600, env=_env(Q2A_BENCH_REHEARSE="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    # (gloo prints its rendezvous notes to stdout; the bench's result is the one JSON line)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2"
    assert res["config"]["global_batch"] == 4 and res["scaling"] == "weak"
    assert res["value"] > 0 and res["steps"] == 2
    assert res["setup_s"]["weight_h2d_plus_rccl_broadcast"] > 0


@pytest.mark.gpu
def test_bench_rccl_world_size_one(tmp_path):
    """The driver's own launch form (`torch.distributed.run --nproc-per-node N ... bench.py --gpus N`) at N = 1 with the
    process group forced up (Q2A_BENCH_PG=1): the RCCL communicator is created on the device and the N>1 path's
    collectives run through it (size + blob broadcast on device memory, barriers, the max-over-ranks all-reduce).
    A 1-GPU box cannot run 2 RCCL ranks (one device per rank), so this is the most of the RCCL path it can execute;
    the engine must come up from the broadcast blob and report one JSON line labelled nccl / dp1."""
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "1", "--steps", "2",
           "--warmup", "1", "--clips", "2", "--config", "f16x1", "--no-cpu-baseline", "--no-host-legs",
           "--workdir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=_env(Q2A_BENCH_PG="1"))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["setup_s"]["collective_backend"] == "nccl"
    assert res["n_gpus"] == 1 and res["config"]["parallelism"] == "dp1" and res["value"] > 0
    assert res["setup_s"]["weight_h2d_plus_rccl_broadcast"] > 0


def test_bench_constants_and_profile_selection():
    """CPU-only: the bench's algorithmic work per clip is SURVEY.md §8d's (2 273.77 GFLOP; weight GEMMs 1 887.44,
    fc1 19.66 per layer), and the committed PMC / SQ summaries it cites are the PROFILE_TAG set, which must exist for
    the default workload (tags do not sort by date)."""
    sys.path.insert(0, ROOT)
    import bench
    assert abs(bench.FLOP_PER_CLIP / 1e9 - 2273.77) < 0.01
    assert abs(bench.FLOP_WEIGHT_GEMMS_PER_CLIP / 1e9 - 1887.44) < 0.01
    assert abs(bench.FLOP_FC1_PER_CLIP / 1e9 - 19.6608) < 1e-6
    names = os.listdir(os.path.join(ROOT, "profiles"))
    for suffix in ("_q4k64_pmc_traffic.json", "_q4k64_sq_mfma.json"):
        picked = bench._profile_files(f for f in names if f.endswith(suffix))[-1]
        assert picked == bench.PROFILE_TAG + suffix, picked
        with open(os.path.join(ROOT, "profiles", picked)) as f:
            kernels = json.load(f)["kernels"]
        if "pmc" in suffix:
            assert kernels["gemm_fc1"]["hbm_bytes_per_launch_corrected"] > 1.24e9   # >= the algorithmic bytes
        else:
            assert any(e.get("class") == "gemm_fc1" and 0 < e["mfma_busy_frac"] < 1 for e in kernels.values())


def test_roofline_objects_name_the_dominant_kernel():
    """CPU-only: the line's `roofline` is built for whichever matrix-core class dominates the step (attention at the
    default workload), with its algorithmic flops per launch, issued-term figures for the F32-class attention, and
    its PMC traffic / SQ busy from the committed summaries of that workload; fc1 keeps its own object."""
    sys.path.insert(0, ROOT)
    import bench
    ms, n = [0.0] * 11, [0] * 11
    ms[5], n[5] = 32 * 1.75 * 3, 32 * 3          # 1.75 ms per attention launch
    ms[8], n[8] = 32 * 1.30 * 3, 32 * 3
    r = bench.roofline_of(5, ms, n, "q4k64", "q4_k", False, 64)
    flop = 4.0 * 1500 * 1500 * 1280 * 64
    assert r["flop_per_launch"] == flop and abs(r["achieved"] - flop / 1.75e-3 / 1e12) < 0.1
    assert abs(r["issued_tflops"] - 3 * r["achieved"]) < 0.5 and "k_attn_t" in r["kernel"]
    assert r["traffic"] and r["traffic"] > 1e9 and r["mfma_busy_frac"] and 0 < r["mfma_busy_frac"] < 1
    f = bench.roofline_of(8, ms, n, "q4k64", "q4_k", False, 64)
    assert f["flop_per_launch"] == 2.0 * 96000 * 5120 * 1280 and "PRE_H,256,2" in f["kernel"]
    assert bench.roofline_of(5, ms, n, "q4k64", "q4_k", False, 2)["traffic"] is None   # other batch: no counters


def test_pmc_summary_splits_o_and_fc2_by_dispatch_order(tmp_path):
    """CPU-only: profiles/pmc_summary.py gives O and fc2 their own traffic although they share the residual-epilogue
    kernels — per layer O first, then fc2's main rounds and (64 clips) its 128x128 partial-round tail."""
    sys.path.insert(0, os.path.join(ROOT, "profiles"))
    import pmc_summary
    main = "void (anonymous namespace)::k_gemm<256, 256, 2, 4, 1, 256, 1>(q2a_gemm_args)"
    tail = "void (anonymous namespace)::k_gemm<128, 128, 2, 2, 1, 256, 0>(q2a_gemm_args)"
    other = "void (anonymous namespace)::k_gemm<256, 256, 2, 4, 7, 256, 2>(q2a_gemm_args)"
    seq = [(other, 5.0), (main, 10.0), (main, 40.0), (tail, 4.0), (other, 5.0), (main, 12.0), (main, 44.0), (tail, 6.0)]
    paths = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        p = tmp_path / f"{counter}.csv"
        with open(p, "w") as f:
            f.write('"Dispatch_Id","Kernel_Name","Counter_Name","Counter_Value"\n')
            for i, (k, v) in enumerate(seq):
                f.write(f'{i + 1},"{k}","{counter}",{v}\n')
        paths[counter] = str(p)
    o, fc2 = pmc_summary.resid_split(paths["FETCH_SIZE"], "FETCH_SIZE")
    assert o == [10.0, 12.0] and fc2 == [44.0, 50.0]
    out = tmp_path / "s.json"
    sys.argv = ["pmc_summary.py", paths["FETCH_SIZE"], paths["WRITE_SIZE"], str(out), "test"]
    pmc_summary.main()
    k = json.load(open(out))["kernels"]
    assert k["gemm_o"]["hbm_bytes_per_launch_corrected"] == (2 * 11.0 + 11.0) * 1024
    assert k["gemm_fc2"]["hbm_bytes_per_launch_corrected"] == (2 * 47.0 + 47.0) * 1024


def test_step_mfma_util_from_the_committed_profile_set():
    """CPU-only: the bench line's `mfma_util` (the metric's "MFMA util %" over a whole step) comes from the committed
    PROFILE_TAG set of the workload — SQ busy per kernel x rocprofv3 time per step / step time — for the BASELINE
    configs and the 64-clip F16 / one-clip Q4_K lines (the exact-Q8_0 q80x64 extra has no set: its line carries null)."""
    sys.path.insert(0, ROOT)
    import bench
    for config in ("q4k64", "f16x1", "q80bf16x64", "f16x64", "q4kx1"):
        u = bench.mfma_util_of(config, bench.CONFIGS[config][1])
        assert u is not None, config
        assert 0.1 < u["value"] < 0.9, (config, u)
        assert all(src.startswith(f"profiles/{bench.PROFILE_TAG}_{config}_") for src in u["sources"]), u
    assert bench.mfma_util_of("q4k64", 3) is None   # another batch than the profiled one: no figure
