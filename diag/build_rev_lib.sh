#!/bin/bash
# build libq2a.so of a git revision into diag/<name>/libq2a.so (A/B timing against the working tree on one box)
set -e
REV=$1; NAME=$2
WT=/tmp/q2a_wt_$NAME
rm -rf $WT; git -C /root/repo worktree prune
git -C /root/repo worktree add -f --detach $WT $REV > /dev/null
make -C $WT/qwen2-audio-whisper-ggml_amd -j8 lib/libq2a.so > /dev/null
mkdir -p /root/repo/diag/$NAME
cp $WT/qwen2-audio-whisper-ggml_amd/lib/libq2a.so /root/repo/diag/$NAME/libq2a.so
git -C /root/repo worktree remove --force $WT
echo built diag/$NAME/libq2a.so from $REV
