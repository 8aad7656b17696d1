# kernel + memory-copy trace of the registered stored-bytes pipeline (tools/e2e_pipe_probe.py --register)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/e2e_trace
mkdir -p $O
timeout -k 10 300 python3 tools/e2e_pipe_probe.py --register 4 6 8 > $O/probe.txt 2>&1 || { tail $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o kt --output-format csv -- \
  python3 tools/e2e_pipe_probe.py --register 6 > $O/kt_probe.txt 2> $O/kt.err || { tail $O/kt.err; exit 1; }
python3 tools/e2e_timeline.py $O/kt 24 > $O/timeline.txt && cat $O/timeline.txt
