#!/bin/bash
# round 6 closing set after the late-round load fixes, parts B and D in one call (tag r06ad): see gpurun_r06ad2.sh and
# gpurun_r06ad4.sh
cd /root/repo
bash diag/gpurun_r06ad2.sh || exit 1
bash diag/gpurun_r06ad4.sh || exit 1
