#!/bin/bash
# round 6: the reference's whisper_full on the ggml backend (one full-size clip, F16 and Q4_K) with rocprofv3 kernel
# traces, to attribute the backend's encode against the engine's one-clip encode (profiles/r06j_f16x1_*)
cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
GB_PROF=1 timeout -k 10 900 bash diag/ggml_backend_timing.sh > gpurun_out/r06l_gb.log 2>&1 || { tail -20 gpurun_out/r06l_gb.log; exit 1; }
cat gpurun_out/r06l_gb.log
find gpurun_out/gb_prof_f16 gpurun_out/gb_prof_q4_k -name "*stats*"
echo done
