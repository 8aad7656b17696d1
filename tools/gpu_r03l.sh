# host-side HIP API trace of the e2e pipeline (K = 4): which call blocks between chunk uploads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $O/ht -o ht --output-format csv -- python3 tools/e2e_pipe_probe.py 4 > $O/ht.txt 2>&1 || { echo HTFAIL; tail $O/ht.txt; exit 1; }
ls $O/ht
