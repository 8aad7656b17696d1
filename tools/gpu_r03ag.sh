# staged TPraos: new equivalence test + TPraos tests, tp bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_tpraos.py > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --config tp --steps 10 > $O/tp.json 2> $O/tp.err || { echo BENCHFAIL; tail $O/tp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/tp.json'));r=d['roofline'];print(d['value'],d['ms_per_step'],r['kernel'],r['frac'],r.get('frac_of_issue_weighted'),r['work_per_unit'])"
