#!/bin/bash
# round 3: k_attn_t with and without its sched_group_barrier interleaving (diag/attn_nosched), same box, two reps
# (diag/attn_t0), alternating, two reps, then one SQ pass (bank conflicts) over the product's attention
cd /root/repo
mkdir -p gpurun_out
export Q2A_BENCH_DIR=/tmp/q2ab Q2A_PARITY_LOG=$PWD/gpurun_out/n_parity_log.jsonl
s() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); pk=d['per_kernel']
print(sys.argv[1], d['ms_per_step'], 'attn', pk['attention']['ms_per_step'])" $1; }
L=qwen2-audio-whisper-ggml_amd/lib/libq2a.so
for i in 1 2; do
for v in new=$L ns=diag/attn_nosched/libq2a.so; do
  n=${v%%=*}; lib=${v#*=}
  Q2A_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-legs > gpurun_out/n_b_$n$i.json 2> gpurun_out/n_b_$n$i.err && s gpurun_out/n_b_$n$i.json || { tail -20 gpurun_out/n_b_$n$i.err; exit 1; }
done
done
O=$PWD/gpurun_out/n_sq
mkdir -p $O
( cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_attn" -d $O -o run --output-format csv -- python3 /root/repo/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-legs > /dev/null 2> $O/err.txt ) || exit 1
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('/root/repo/gpurun_out/n_sq/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(float); n = collections.Counter()
for r in csv.DictReader(open(f)):
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']] += 1
print({k: acc[k] / max(1, n[k]) for k in acc}, 'rows per counter', dict(n))
PY
