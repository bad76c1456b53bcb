#!/bin/bash
# round 6: which cross-lane form for the LayerNorm kernels (all three bit-identical, checked first): nowpe = LDS-pipe
# (ds_bpermute) f64 sums and Q8_K reductions; mixA = LDS-pipe f64 sums, Q8_K max / bsum on DPP; new = everything on
# DPP / permlane swaps (+ the 64-VGPR cap). Alternating 64-clip benches on one box.
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
lib() { case $1 in new) unset Q2A_LIB_PATH;; *) export Q2A_LIB_PATH=$PWD/diag/$1/libq2a.so;; esac; }
for v in nowpe mixA new; do
  lib $v
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06y_bits_$v.json 2> gpurun_out/r06y_err.log || { tail -5 gpurun_out/r06y_err.log; exit 1; }
done
python3 - <<'E' || exit 1
import json
a, b, c = (json.load(open(f"gpurun_out/r06y_bits_{v}.json")) for v in ("nowpe", "mixA", "new"))
same = {k: a[k] == b[k] == c[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
run() {  # config variant rep
  lib $2
  timeout -k 10 300 python3 bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06y_$1_$2_$3.json 2> gpurun_out/r06y_err.log || { tail -5 gpurun_out/r06y_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06y_$1_$2_$3.json'));print('$1 $2 $3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm', 'quant_act')})"
}
for i in 1 2 3; do for v in nowpe mixA new; do run q4k64 $v $i || exit 1; done; done
for i in 1 2; do for v in nowpe mixA new; do run f16x64 $v $i || exit 1; done; done
echo done
