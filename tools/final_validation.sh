#!/bin/bash
# Round-end validation on one GPU box (gpurun): GPU suite, smoke, PMC traffic of this library (installed as
# profiles/pmc_traffic.json so the bench prices its roofline with it), the bench line, rocprofv3 kernel stats of the
# pipelined and the sequential step.  usage: TAG=<name> bash tools/final_validation.sh  (outputs under gpurun_out/<name>)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${TAG:-final}
O=gpurun_out/$T; mkdir -p $O
echo "lib $(python3 -c 'import sys; sys.path.insert(0,"3d_multiview_reg_amd"); from lib import _native; print(_native.source_hash())')"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_suite.log 2>&1 || { tail -30 $O/gpu_suite.log; exit 1; }
tail -1 $O/gpu_suite.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
echo smoke ok
bash tools/pmc_bench.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_traffic.py $O/pmc --out $O/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || { tail -20 $O/pmc_traffic.log; exit 1; }
cp $O/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -c 600 $O/bench.log
bash tools/prof_bench.sh $O/prof_pipe --no-secondary > $O/prof_pipe.log 2>&1 || { tail -20 $O/prof_pipe.log; exit 1; }
bash tools/prof_bench.sh $O/prof_seq --no-pipeline --no-secondary --steps 7 --warmup 2 > $O/prof_seq.log 2>&1 || { tail -20 $O/prof_seq.log; exit 1; }
echo done
