#!/bin/bash
# r9g: prompt processing (64 x 512-token prompts, exact mode) on the final round-4 build: 70B Q4_K and
# 8B Q4_K_M, the default prompt chunk and 2048-token chunks
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
P="timeout -k 10 300 python3 tools/prefill_bench.py"
$P > $O/r9g_70.log 2>&1 || { tail -3 $O/r9g_70.log; exit 1; }; echo "70b: $(tail -1 $O/r9g_70.log)"
$P --set prefill_chunk=2048 > $O/r9g_70c.log 2>&1 || { tail -3 $O/r9g_70c.log; exit 1; }; echo "70b chunk 2048: $(tail -1 $O/r9g_70c.log)"
$P --model llama3-8b --ftype Q4_K_M > $O/r9g_8.log 2>&1 || { tail -3 $O/r9g_8.log; exit 1; }; echo "8b: $(tail -1 $O/r9g_8.log)"
$P --model llama3-8b --ftype Q4_K_M --set prefill_chunk=2048 > $O/r9g_8c.log 2>&1 || { tail -3 $O/r9g_8c.log; exit 1; }; echo "8b chunk 2048: $(tail -1 $O/r9g_8c.log)"
