#!/bin/bash
# r11d: gemvs timing probes on the 8B single-stream shapes (tools/gemvs_probe.hip, built on the CPU side into bin/):
# GEMVS_PROBE 0 real, 1 no dequant/MFMA, 2 no x prologue, 3 = 1+2, 4 plain store, 7 all
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O
timeout -k 10 300 $R/distributed-llm-pipeline_amd/bin/gemvs_probe > $O/r11d_gemvs_probe.txt 2>&1; rc=$?; cat $O/r11d_gemvs_probe.txt; exit $rc
