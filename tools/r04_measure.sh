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
echo MEASURE_DONE
