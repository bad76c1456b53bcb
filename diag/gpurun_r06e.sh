#!/bin/bash
# round 6: whole GPU suite with the whole-line register-path epilogue stores (every non-staged fp16 / f32 epilogue)
# and the row-major V operand of the reference-contract attention (k_attn_t<true>) and the persistent Q4_K Q|K|V GEMM,
# configs[1] NULL vs explicit stream, then the stores A/B against the previous epilogue (diag/regbase), alternating
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06e_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -4 gpurun_out/r06e_tests.log
case $rc in 0) ;; *) exit 1;; esac
rm -f gpurun_out/r06d_null_stream.jsonl
for c in f16x1 q4kx1; do
  timeout -k 10 300 python3 diag/null_stream_ab.py $c >> gpurun_out/r06d_null_stream.jsonl 2> gpurun_out/r06e_err.log || { tail -5 gpurun_out/r06e_err.log; exit 1; }
done
cat gpurun_out/r06d_null_stream.jsonl
for c in f16x1 q4kx1 f16x64 q4k64; do
  for i in 1 2; do
    for v in base new; do
      if [ $v = base ]; then export Q2A_LIB_PATH=$PWD/diag/regbase/libq2a.so; else unset Q2A_LIB_PATH; fi
      timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-host-legs > gpurun_out/r06e_${c}_${v}_$i.json 2> gpurun_out/r06e_err.log || { tail -5 gpurun_out/r06e_err.log; exit 1; }
      python3 -c "import json;d=json.load(open('gpurun_out/r06e_${c}_${v}_$i.json'));print('$c $v $i', d['ms_per_step'], {k: v['ms_per_step'] for k, v in d['per_kernel'].items() if k.startswith('gemm') or k.startswith('conv')})"
    done
  done
done
