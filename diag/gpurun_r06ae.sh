#!/bin/bash
# round 6: LayerNorm + Q8_K of the model-width rows two rows per wave (k_ln_q8k_2rows: both rows' loads in flight, the
# two reduction chains interleaved, 16 rows per workgroup) against one row per wave (diag/ln1base = k_rownorm5):
# output bits, then alternating benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
lib() { case $1 in new) unset Q2A_LIB_PATH;; *) export Q2A_LIB_PATH=$PWD/diag/$1/libq2a.so;; esac; }
for v in new ln1base; do
  lib $v
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06ae_bits_$v.json 2> gpurun_out/r06ae_err.log || { tail -5 gpurun_out/r06ae_err.log; exit 1; }
done
python3 - <<'E' || exit 1
import json
a, b = (json.load(open(f"gpurun_out/r06ae_bits_{v}.json")) for v in ("new", "ln1base"))
same = {k: a[k] == b[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
run() {  # config variant rep
  lib $2
  timeout -k 10 300 python3 bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06ae_$1_$2_$3.json 2> gpurun_out/r06ae_err.log || { tail -5 gpurun_out/r06ae_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06ae_$1_$2_$3.json'));print('$1 $2 $3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm',)})"
}
for i in 1 2 3; do for v in new ln1base; do run q4k64 $v $i || exit 1; done; done
for v in new ln1base; do run q4kx1 $v 1 || exit 1; done
echo done
