#!/bin/bash
# round 6 closing set after the late-round load fixes, part A (tag r06ad): output bits against the library before the
# k_pool_ln load change (diag/plbase), whole GPU suite + smoke, the default bench line (CPU baseline, c_group leg), then
# rocprofv3 kernel stats + PMC traffic for configs[1]
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab
for v in plbase new; do
  if [ $v = plbase ]; then export Q2A_LIB_PATH=$PWD/diag/plbase/libq2a.so; else unset Q2A_LIB_PATH; fi
  timeout -k 10 600 python3 diag/lib_bits.py > gpurun_out/r06ad_bits_$v.json 2> gpurun_out/r06ad_err.log || { tail -5 gpurun_out/r06ad_err.log; exit 1; }
done
unset Q2A_LIB_PATH
python3 - <<'E' || exit 1
import json
a, b = (json.load(open(f"gpurun_out/r06ad_bits_{v}.json")) for v in ("plbase", "new"))
same = {k: a[k] == b[k] for k in a if k != "lib"}
print("bits identical:", same)
assert all(same.values())
E
Q2A_PARITY_LOG=$PWD/gpurun_out/r06ad_parity_log.jsonl timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r06ad_tests.log 2>&1; rc=$?
echo "gpu tests rc=$rc"; tail -3 gpurun_out/r06ad_tests.log
case $rc in 0) ;; *) exit 1;; esac
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06ad_smoke.log 2>&1 || { tail -5 gpurun_out/r06ad_smoke.log; exit 1; }
tail -1 gpurun_out/r06ad_smoke.log
timeout -k 10 900 python3 bench.py > gpurun_out/r06ad_bench_q4k64.json 2> gpurun_out/r06ad_bench.err || { tail -5 gpurun_out/r06ad_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r06ad_bench_q4k64.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_gemm_fc1']['frac'], d['cpu_baseline']['value'], d['c_group'])"
timeout -k 10 900 bash profiles/collect.sh r06ad f16x1 > gpurun_out/r06ad_collect.log 2>&1 || { tail -5 gpurun_out/r06ad_collect.log; exit 1; }
echo done
