#!/bin/bash
# round 5: the first attention's operands, fused Q|K|V route vs separate projections (full F16), compared per array
cd /root/repo
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
H=oracle/_ref/ggml_harness
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null
$T synth-clip $W/clip0.f32 480000 0 > /dev/null
export LD_LIBRARY_PATH=$PWD/diag/dump
Q2A_DUMP_ATTN=$W/d_fused.bin timeout -k 10 120 $H encode $W/full-f16.bin $W/clip0.f32 $W/o1.f32 1 > /dev/null || exit 1
Q2A_DUMP_ATTN=$W/d_sep.bin GGML_Q2A_NO_FUSED_QKV=1 timeout -k 10 120 $H encode $W/full-f16.bin $W/clip0.f32 $W/o2.f32 1 > /dev/null || exit 1
python3 - <<'PY'
import numpy as np
W='/tmp/q2a_gb'
a=np.fromfile(W+'/d_fused.bin',dtype=np.float16); b=np.fromfile(W+'/d_sep.bin',dtype=np.float16)
T,D,TP=1500,1280,1536
nq=T*D; nv=D*TP
print('sizes', a.size, b.size)
names=['qh','ql','kh','kl','vt','vtl']; offs=[0,nq,2*nq,3*nq,4*nq,4*nq+nv]; lens=[nq]*4+[nv]*2
for n,o,l in zip(names,offs,lens):
    x=a[o:o+l].astype(np.float32); y=b[o:o+l].astype(np.float32)
    ne=int((a[o:o+l].view(np.uint16)!=b[o:o+l].view(np.uint16)).sum())
    idx=np.nonzero(a[o:o+l].view(np.uint16)!=b[o:o+l].view(np.uint16))[0][:8]
    print(n, 'differ', ne, 'maxabs', float(np.abs(x-y).max()), 'first', idx.tolist(), x[idx].tolist(), y[idx].tolist())
qf=np.fromfile(W+'/d_fused.bin.q',dtype=np.float32); qs=np.fromfile(W+'/d_sep.bin.q',dtype=np.float32)
print('Q f32 sizes', qf.size, qs.size, 'differ', int((qf.view(np.uint32)!=qs.view(np.uint32)).sum()))
d=np.nonzero(qf.view(np.uint32)!=qs.view(np.uint32))[0][:8]
print('first', d.tolist(), qf[d].tolist(), qs[d].tolist())
L=np.float32(1.4426950408889634)
vs=qs*L; hs=vs.astype(np.float16)
qh=a[0:nq]
print('sep hi from dumped Q == dumped sep qh:', int((hs.view(np.uint16)!=b[0:nq].view(np.uint16)).sum()))
vf=qf*L; hf=vf.astype(np.float16)
print('hi from fused-store Q vs fused qh:', int((hf.view(np.uint16)!=qh.view(np.uint16)).sum()))
PY
