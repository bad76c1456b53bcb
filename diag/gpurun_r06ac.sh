#!/bin/bash
# round 6: the log-mel frame kernel issues a frame's input loads together (clamped addresses, then the reflect / range
# selects) against the previous library (diag/melbase): mel bit-exactness tests, output bits, alternating benches
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "mel or short_audio or batch_equals" --timeout 300 --timeout-method thread > gpurun_out/r06ac_tests.log 2>&1; rc=$?
tail -2 gpurun_out/r06ac_tests.log
case $rc in 0) ;; *) exit 1;; esac
lib() { case $1 in new) unset Q2A_LIB_PATH;; *) export Q2A_LIB_PATH=$PWD/diag/$1/libq2a.so;; esac; }
for v in melbase new; do
  lib $v
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06ac_bits_$v.json 2> gpurun_out/r06ac_err.log || { tail -5 gpurun_out/r06ac_err.log; exit 1; }
done
python3 - <<'E' || exit 1
import json
a, b = (json.load(open(f"gpurun_out/r06ac_bits_{v}.json")) for v in ("melbase", "new"))
same = {k: a[k] == b[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
run() {  # config variant rep
  lib $2
  timeout -k 10 300 python3 bench.py --config $1 --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06ac_$1_$2_$3.json 2> gpurun_out/r06ac_err.log || { tail -5 gpurun_out/r06ac_err.log; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/r06ac_$1_$2_$3.json'));print('$1 $2 $3', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('mel',)})"
}
for i in 1 2; do for c in f16x1 q4k64; do for v in melbase new; do run $c $v $i || exit 1; done; done; done
echo done
