cd /root/repo && mkdir -p gpurun_out && export TMPDIR=/tmp
W=/tmp/q2a_gb; mkdir -p $W
T=qwen2-audio-whisper-ggml_amd/bin/q2a_tool
$T gen-model $W/full-f16.bin full f16 0x51A2 16 > /dev/null && $T synth-clip $W/clip0.f32 480000 0 > /dev/null || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06n_prof -o gb --output-format csv -- oracle/_ref/ggml_harness encode $W/full-f16.bin $W/clip0.f32 $W/o.f32 8 > gpurun_out/r06n_prof.json 2> gpurun_out/r06n_prof.err || { tail -5 gpurun_out/r06n_prof.err; exit 1; }
find gpurun_out/r06n_prof -name "*kernel_stats.csv"
