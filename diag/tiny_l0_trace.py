"""Layer-0 divergence of the tiny F16 model, engine vs the reference's builds (diagnostic).

  python diag/tiny_l0_trace.py ref OUT.npz      (build container: every oracle/_ref* build, clip 0, layer-0 dumps)
  python diag/tiny_l0_trace.py gpu REF.npz      (GPU box: the engine's front end + layer 0 through the GEMM taps)

ref: for each reference build, the first-block nodes (3 conv out, 6 LN1, 24 attention, 27 x1, 30 LN2, 33 GELU,
36 x2) of tiny-f16 on clip 0 -> OUT.npz, and the pairwise fp16-code flips / rel-L2 per node between builds.
gpu: the engine's layer-0 values at the points it converts to fp16 for a GEMM (LN1 -> QKV, attention -> O, LN2 ->
fc1, GELU -> fc2) against the AVX2 build's: fp16 codes that differ, rel-L2 of the f32 values where available."""
import glob
import json
import os
import shutil
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "bin", "q2a_tool")
BUILDS = {"avx2": "_ref", "x86-64": "_ref_x86-64", "avx512": "_ref_avx512", "sse42": "_ref_v2", "avx2-fma": "_ref_fma"}
NODES = {3: "conv_out", 6: "ln1", 24: "attn", 27: "x1", 30: "ln2", 33: "gelu", 36: "x2"}


def rel_l2(a, b):
    return float(np.linalg.norm(a.astype(np.float64) - b) / np.linalg.norm(b.astype(np.float64)))


def ref(out):
    work = "/tmp/q2a_l0"
    os.makedirs(work, exist_ok=True)
    model, clip = os.path.join(work, "tiny-f16.bin"), os.path.join(work, "clip0.f32")
    if not os.path.exists(model):
        subprocess.check_call([TOOL, "gen-model", model, "tiny", "f16", "0x51A2", "8"])
    if not os.path.exists(clip):
        subprocess.check_call([TOOL, "synth-clip", clip, "480000", "0"])
    arrs = {}
    for b, d in BUILDS.items():
        dump = os.path.join(work, f"dump-{b}")
        shutil.rmtree(dump, ignore_errors=True)
        os.makedirs(dump)
        subprocess.run([os.path.join(ROOT, "oracle", d, "ref_harness"), "encode", model, clip, os.path.join(dump, "y.f32"),
                        "8", "1", dump, "40"], check=True, capture_output=True)
        for n, nm in NODES.items():
            arrs[f"{b}_{nm}"] = np.fromfile(glob.glob(os.path.join(dump, f"node{n:03d}_*.f32"))[0], dtype=np.float32)
    np.savez(out, **{k: v for k, v in arrs.items() if k.startswith("avx2_")})
    names = list(BUILDS)
    for nm in NODES.values():
        for i, a in enumerate(names):
            for c in names[i + 1:]:
                x, y = arrs[f"{a}_{nm}"], arrs[f"{c}_{nm}"]
                flips = int((x.astype(np.float16) != y.astype(np.float16)).sum())
                print(json.dumps({"node": nm, "pair": f"{a}_vs_{c}", "fp16_flips": flips, "rel_l2": rel_l2(y, x)}))


def gpu(refnpz):
    sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
    import torch
    import q2a
    r = dict(np.load(refnpz))
    work = "/tmp/q2a_l0"
    os.makedirs(work, exist_ok=True)
    model, clip = os.path.join(work, "tiny-f16.bin"), os.path.join(work, "clip0.f32")
    subprocess.check_call([TOOL, "gen-model", model, "tiny", "f16", "0x51A2", "16"])
    subprocess.check_call([TOOL, "synth-clip", clip, "480000", "0"])
    e = q2a.Engine(model, device=0)
    T, D = e.info.n_audio_ctx, e.info.n_audio_state
    pcm = torch.from_numpy(np.fromfile(clip, dtype=np.float32)).cuda()
    x = torch.empty((T, D), dtype=torch.float32, device="cuda")
    e.test_frontend(pcm.data_ptr(), pcm.numel(), [pcm.numel()], x.data_ptr())
    torch.cuda.synchronize()
    conv = x.cpu().numpy().reshape(-1)
    taps = [torch.zeros((T, D), dtype=torch.float16, device="cuda") for _ in range(3)] + \
           [torch.zeros((T, 4 * D), dtype=torch.float16, device="cuda")]
    e.test_block_taps(0, x.data_ptr(), 1, [t.data_ptr() for t in taps])
    torch.cuda.synchronize()
    tp = [t.cpu().numpy().reshape(-1) for t in taps]
    x2 = x.cpu().numpy().reshape(-1)
    print(json.dumps({"node": "conv_out", "rel_l2": rel_l2(conv, r["avx2_conv_out"]),
                      "fp16_flips": int((conv.astype(np.float16) != r["avx2_conv_out"].astype(np.float16)).sum())}))
    for nm, t in zip(("ln1", "attn", "ln2", "gelu"), tp):
        print(json.dumps({"node": nm, "fp16_flips": int((t != r[f"avx2_{nm}"].astype(np.float16)).sum()),
                          "rel_l2_fp16": rel_l2(t.astype(np.float32), r[f"avx2_{nm}"])}))
    print(json.dumps({"node": "x2", "rel_l2": rel_l2(x2, r["avx2_x2"])}))
    e.close()


if __name__ == "__main__":
    (ref if sys.argv[1] == "ref" else gpu)(sys.argv[2])
