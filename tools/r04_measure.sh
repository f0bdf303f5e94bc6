#!/bin/bash
# VERDICT r03 #5/#6 measurements: exchange proxy at N = 8 (full and points)
# and the host-fed ingest rate at depth 1-3, beside the resident bench line.
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --no-cpu --exchange-proxy 8 > $O/m_proxy8.json 2> $O/m_proxy8.err || { tail -20 $O/m_proxy8.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/m_proxy8.json').read().strip().splitlines()[0]);print(d['value'],d['ms_per_step']);print(json.dumps(d['exchange_proxy']))"
timeout -k 10 300 python3 tools/ingest_bench.py --depths 1,2,3 > $O/m_ingest.jsonl 2> $O/m_ingest.err || { tail -20 $O/m_ingest.err; exit 1; }
cat $O/m_ingest.jsonl
timeout -k 10 200 python3 bench.py --batch 1 --steps 200 --warmup 20 --no-cpu > $O/m_config2.json 2> $O/m_config2.err || { tail -20 $O/m_config2.err; exit 1; }
head -c 400 $O/m_config2.json; echo

# config #5: bench line and the describe kernel's SQ counters for the bound model
C5="--batch 64 --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1"
timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu $C5 > $O/m_config5.json 2> $O/m_config5.err || { tail -20 $O/m_config5.err; exit 1; }
head -c 600 $O/m_config5.json; echo
bash tools/pmc.sh c5sq "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" $C5 | grep -E "k_describe" || exit 1
echo MEASURE2_DONE
