#!/bin/bash
# r8n: 8-wave decode attention for small grids (single stream): tests, 8B / 70B mb1 kernel traces vs 4 waves
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
T="timeout -k 10 400 python -u -m pytest -q -x --timeout 250 --timeout-method thread -m gpu -p no:cacheprovider"
$T tests/test_attn_wave_gpu.py tests/test_engine_gpu.py -k "attn or wave or decode or reference or fp8 or single" > $O/r8n_t.log 2>&1; rc=$?; tail -2 $O/r8n_t.log; [ $rc -ne 0 ] && exit $rc
MIPIPE_ATTN_KFL=1 $T tests/test_attn_wave_gpu.py > $O/r8n_tk.log 2>&1; rc=$?; tail -1 $O/r8n_tk.log; [ $rc -ne 0 ] && exit $rc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -Wno-unused-value -Wno-unused-result tools/load_pattern_bench.hip -o /tmp/lpb > $O/r8n_lpb_build.log 2>&1 || { tail -3 $O/r8n_lpb_build.log; exit 1; }
timeout -k 10 120 /tmp/lpb | tee $O/r8n_lpb.log || exit 1
cd /tmp
P="timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -o run"
pr() { local n=$1; shift; $P -d $O/r8n_$n -- python3 $R/bench.py --steps 20 --warmup 2 --no-secondary "$@" > $O/r8n_$n.log 2>&1 || { tail -3 $O/r8n_$n.log; exit 1; }
  python3 $R/tools/prof_summary.py $O/r8n_$n > $O/r8n_$n.txt; echo "== $n $(grep -o '"value": [0-9.]*' $O/r8n_$n.log) $(grep -m2 -E 'attn_decode' $O/r8n_$n.txt | tail -1 | cut -c1-100)"; }
pr 8b_w8 --model llama3-8b --ftype Q4_K_M --mb-size 1
export MIPIPE_ATTN_NW8_MAXWG=0; pr 8b_w4 --model llama3-8b --ftype Q4_K_M --mb-size 1; unset MIPIPE_ATTN_NW8_MAXWG
pr 70b_w8 --mb-size 1
export MIPIPE_ATTN_NW8_MAXWG=0; pr 70b_w4 --mb-size 1; unset MIPIPE_ATTN_NW8_MAXWG
pr 8b_w8_ctx1000 --model llama3-8b --ftype Q4_K_M --mb-size 1 --prompt-len 1000
# whole-line K loads in the wave attention (knob ATTN_KFL): 70B mb256 at 128 and 2K contexts
for kfl in 0 1; do
  export MIPIPE_ATTN_KFL=$kfl
  pr 70b_kfl$kfl
  pr 70b_2k_kfl$kfl --mb-size 64 --prompt-len 1984 --steps 10
done
unset MIPIPE_ATTN_KFL
