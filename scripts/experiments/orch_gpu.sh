#!/bin/bash
# orchestrator on the GPU (synthetic 8B Q4_K_M, 2 emulated stages): /chat SSE, /completion, /health, /metrics
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out; mkdir -p $O; cd $R
B=./distributed-llm-pipeline_amd/bin
timeout -k 5 150 $B/orchestrator --synthetic llama3-8b --ftype Q4_K_M --stages 2 --devices 0,0 --mb-size 4 -n 24 -c 512 --port 3077 > $O/orch.log 2>&1 &
PID=$!
for i in $(seq 1 60); do curl -s localhost:3077/health > /dev/null 2>&1 && break; sleep 1; done
curl -s -N -m 60 -X POST localhost:3077/chat -H 'Content-Type: application/json' -d '{"prompt":"Once upon a time"}' > $O/orch_chat.txt
echo "chat events: $(grep -c '^data:' $O/orch_chat.txt) (token: $(grep -c '"msg_type":"token"' $O/orch_chat.txt), log: $(grep -c '"msg_type":"log"' $O/orch_chat.txt))"
grep -m3 'offloaded\|RPC\|stage' $O/orch_chat.txt | cut -c1-200
for i in 1 2 3; do curl -s -m 60 -X POST localhost:3077/completion -H 'Content-Type: application/json' -d '{"prompt":"The pipeline","n_predict":16}' > $O/orch_c$i.json & done; wait %2 %3 %4 2>/dev/null
head -c 300 $O/orch_c1.json; echo
curl -s -m 10 localhost:3077/health; echo
curl -s -m 10 localhost:3077/metrics | head -20
kill $PID; wait $PID 2>/dev/null; echo "orchestrator exit: $?"
