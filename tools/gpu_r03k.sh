# e2e pipeline probe: chunk counts, then a kernel + memory-copy trace of K=2 and K=4
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u tools/e2e_pipe_probe.py 2 3 4 6 8 > $O/probe.txt 2>&1 || { echo PROBEFAIL; tail $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt2 -o kt --output-format csv -- python3 tools/e2e_pipe_probe.py 2 > $O/kt2.txt 2>&1 || { echo KT2FAIL; tail $O/kt2.txt; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt4 -o kt --output-format csv -- python3 tools/e2e_pipe_probe.py 4 > $O/kt4.txt 2>&1 || { echo KT4FAIL; tail $O/kt4.txt; exit 1; }
ls -R $O | head -30
