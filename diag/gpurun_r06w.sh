#!/bin/bash
# round 6: the LayerNorm kernels issue all of a row's loads before the sums (they compiled to one load + vmcnt(0) per
# chunk). Output bits of the new library against the previous one (diag/lnbase2, git HEAD before the change) on the
# same box, alternating 64-clip benches (Q4_K: LN + Q8_K; F16: LN + fp16), then the whole GPU suite
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for v in base new; do
  if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/lnbase2/libq2a.so; else unset Q2A_LIB_PATH; fi
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06w_bits_$v.json 2> gpurun_out/r06w_err.log || { tail -5 gpurun_out/r06w_err.log; exit 1; }
done
python3 - <<'E' || exit 1
import json
a, b = (json.load(open(f"gpurun_out/r06w_bits_{v}.json")) for v in ("base", "new"))
same = {k: a[k] == b[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
for c in q4k64 f16x64; do
  for i in 1 2; do
    for v in base new; do
      if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/lnbase2/libq2a.so; else unset Q2A_LIB_PATH; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06w_${c}_${v}_$i.json 2> gpurun_out/r06w_err.log || { tail -5 gpurun_out/r06w_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06w_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k in ('layernorm', 'quant_act')})"
    done
  done
done
unset Q2A_LIB_PATH
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06w_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06w_tests.log
echo done
