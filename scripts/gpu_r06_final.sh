#!/bin/bash
# r06 closing session on the final tree: smoke(), the whole GPU suite, the headline profile (scripts/profile.sh) and the
# default bench line. Each step time-limited; a failure ends the session. Usage: bash scripts/gpu_r06_final.sh <tag>
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 10
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 11
bash scripts/profile.sh $TAG || exit 12
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 13
echo done > $O/done.txt
