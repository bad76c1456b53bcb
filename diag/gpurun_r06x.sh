#!/bin/bash
# round 6: LayerNorm rows of D = 1280 with a compile-time row length for every output mode (k_rownorm5: 8 rows per
# 512-thread workgroup, the LayerNorm weight / bias staged in LDS once per workgroup, at most 64 VGPRs) against the
# previous library (diag/lnbase2) and the same kernels without the 64-VGPR cap and with LDS-pipe reductions (diag/nowpe;
# "new" = the cap + every LayerNorm / Q8_K cross-lane step on DPP / permlane swaps): output bits, alternating
# 64-clip benches of every LN mode (Q4_K: Q8_K, F16: fp16, Q8_0: Q8_0, Q8_0 + bf16: bf16), then the whole GPU suite
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
lib() { case $1 in base) export Q2A_LIB_PATH=$PWD/diag/lnbase2/libq2a.so;; nowpe) export Q2A_LIB_PATH=$PWD/diag/nowpe/libq2a.so;; *) unset Q2A_LIB_PATH;; esac; }
for v in base nowpe new; do
  lib $v
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06x_bits_$v.json 2> gpurun_out/r06x_err.log || { tail -5 gpurun_out/r06x_err.log; exit 1; }
done
python3 - <<'E' || exit 1
import json
a, b, c = (json.load(open(f"gpurun_out/r06x_bits_{v}.json")) for v in ("base", "nowpe", "new"))
same = {k: a[k] == b[k] == c[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
run() {  # config variant rep
  lib $2
  timeout -k 10 300 python3 bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06x_$1_$2_$3.json 2> gpurun_out/r06x_err.log || { tail -5 gpurun_out/r06x_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06x_$1_$2_$3.json'));print('$1 $2 $3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm', 'quant_act')})"
}
for i in 1 2; do for v in base nowpe new; do run q4k64 $v $i || exit 1; done; done
for i in 1 2; do for v in base new; do run f16x64 $v $i || exit 1; done; done
for c in q80x64 q80bf16x64; do for v in base new; do run $c $v 1 || exit 1; done; done
unset Q2A_LIB_PATH
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06x_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06x_tests.log
echo done
