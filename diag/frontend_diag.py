"""Front-end divergence of the tiny F16 model on clip 0, engine vs the reference's builds (diagnostic, GPU box).

    python diag/frontend_diag.py REF.npz      (REF.npz: <build>_n3 = node003 (conv out + pe) of each reference build,
                                                made in the build container from oracle/_ref*/ref_harness dumps)
Prints: the GPU log-mel against the oracle's (bit-identical fraction, max |diff|), and the engine's layer-0 input
against every build (exactly equal fraction, fp16-code flips, rel-L2)."""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
TOOL = os.path.join(ROOT, "qwen2-audio-whisper-ggml_amd", "bin", "q2a_tool")


def main(refnpz):
    import torch
    import q2a
    import oracle_py
    from q2a import ggmlfile
    r = dict(np.load(refnpz))
    work = "/tmp/q2a_fe"
    os.makedirs(work, exist_ok=True)
    model, clip = os.path.join(work, "tiny-f16.bin"), os.path.join(work, "clip0.f32")
    subprocess.check_call([TOOL, "gen-model", model, "tiny", "f16", "0x51A2", "16"])
    subprocess.check_call([TOOL, "synth-clip", clip, "480000", "0"])
    pcm = np.fromfile(clip, dtype=np.float32)
    e = q2a.Engine(model, device=0)
    mel = e.pcm_to_mel(pcm)
    orc = oracle_py.Oracle(ggmlfile.read(model)).log_mel(pcm)
    print(json.dumps({"what": "mel", "n": int(mel.size), "bit_equal_frac": float((mel == orc).mean()),
                      "max_abs": float(np.abs(mel.astype(np.float64) - orc).max())}))
    T, D = e.info.n_audio_ctx, e.info.n_audio_state
    pd = torch.from_numpy(pcm).cuda()
    x = torch.empty((T, D), dtype=torch.float32, device="cuda")
    e.test_frontend(pd.data_ptr(), pd.numel(), [pd.numel()], x.data_ptr())
    torch.cuda.synchronize()
    xe = x.cpu().numpy().reshape(-1)
    for k in sorted(r):
        if not k.endswith("_n3"):
            continue
        y = r[k]
        print(json.dumps({"what": "layer0_input", "vs": k[:-3], "exact_frac": float((xe == y).mean()),
                          "fp16_flips": int((xe.astype(np.float16) != y.astype(np.float16)).sum()),
                          "rel_l2": float(np.linalg.norm(xe.astype(np.float64) - y) / np.linalg.norm(y))}))
    e.close()


if __name__ == "__main__":
    main(sys.argv[1])
