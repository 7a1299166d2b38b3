#!/bin/bash
# r11b: stream_probe -- cost of a graph-captured chain of cold weight-streaming kernels by size / grid / depth
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 $R/tools/stream_probe.hip -o /tmp/sp && timeout -k 10 300 /tmp/sp > $O/r11b_stream_probe.txt 2>&1; rc=$?; cat $O/r11b_stream_probe.txt; exit $rc
