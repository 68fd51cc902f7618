set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/c5
timeout -k 10 300 python -u tools/cfg5_leg.py > gpurun_out/c5/leg.json
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/c5/f -o fetch --output-format csv -- python3 tools/cfg5_leg.py > gpurun_out/c5/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/c5/w -o write --output-format csv -- python3 tools/cfg5_leg.py > gpurun_out/c5/w.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/c5/k -o kt --output-format csv -- python3 tools/cfg5_leg.py > gpurun_out/c5/k.log 2>&1
