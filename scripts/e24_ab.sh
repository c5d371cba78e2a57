cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/e24_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/e24_tests.log | head -20; tail -3 gpurun_out/e24_tests.log; exit 1; }
tail -1 gpurun_out/e24_tests.log
for rep in 1 2 3; do
  for cfg in C2 C4 C3; do
    for v in e24 e32; do
      env=; [ $v = e32 ] && env="OCTVR_ENTRY32=1"
      env $env timeout -k 10 240 python bench.py --config $cfg --no-cpu-baseline --no-async-e2e > gpurun_out/e24ab_${v}_${cfg}_$rep.log 2>&1 || { echo "$v $cfg rc=$?"; tail -5 gpurun_out/e24ab_${v}_${cfg}_$rep.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/e24ab_${v}_${cfg}_$rep.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v $cfg $rep', d['value'], d['ms_per_step'], r['kernel_us'], r['bytes_per_launch'])"
    done
  done
done
echo done
