#!/bin/bash
# round-4 GPU batch: new tests first, then the whole -m gpu suite, then short bench legs.
# usage: tools/gpu_r4.sh <tag> [stage...]   stages: new all bench c3 prof
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
export PYTHONUNBUFFERED=1
for st in "$@"; do
  case $st in
    jvp)
      timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_jvp.py tests/test_gpu_metric_parity.py tests/test_gpu_modules.py -s > $out/jvp_tests.txt 2>&1 || exit $? ;;
    fwd)
      timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_fwdreg.py tests/test_gpu_fused.py tests/test_gpu_freg_magic.py tests/test_gpu_wide.py tests/test_gpu_metric_parity.py -s > $out/fwd_tests.txt 2>&1 || exit $? ;;
    stack)
      timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_siren_stack.py -s > $out/stack_tests.txt 2>&1 || exit $? ;;
    new)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gpu_sincos.py tests/test_gpu_jvp.py tests/test_gpu_ddp2.py -s > $out/new_tests.txt 2>&1 || exit $? ;;
    floss)
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
        tests/test_gpu_fused_loss.py tests/test_gpu_kspace.py tests/test_gpu_loss.py tests/test_gpu_modules.py -s > $out/floss_tests.txt 2>&1 || exit $? ;;
    c4)
      timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --no-psnr --no-other-configs > $out/c4.json 2> $out/c4.err || exit $? ;;
    all)
      timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $out/all_tests.txt 2>&1 || exit $? ;;
    bench)
      timeout -k 10 400 python -u bench.py > $out/bench.json 2> $out/bench.err || exit $? ;;
    benchm)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr --no-other-configs > $out/benchm.json 2> $out/benchm.err || exit $? ;;
    c3)
      timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline --no-psnr --no-other-configs > $out/c3.json 2> $out/c3.err || exit $? ;;
    c3prof)
      (cd /tmp && export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/c3prof -o c3 -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --no-cpu-baseline --no-psnr --no-other-configs --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$out/c3prof.log 2>&1) || exit $? ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp; timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o m -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-psnr --no-other-configs --steps 20 --warmup 5 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1) || exit $? ;;
    probe)
      timeout -k 10 300 build/probe_store_hazard > $out/probe_store_hazard.txt 2>&1 || exit $? ;;
  esac
done
