#!/bin/bash
# Runs ON the GPU box (gpurun): one batch of round-5 measurements, every GPU step under its own
# time limit, stopping at the first failure.  Output under gpurun_out/r05/<tag>/.
# usage: tools/r05_batch.sh <tag> <step>...   steps: hash, tests, alltests, c3, c5
set -u
TAG=$1; shift
OUT=gpurun_out/r05/$TAG
mkdir -p $OUT
for step in "$@"; do
    case $step in
    hash)
        timeout -k 10 600 python -u tools/hash_ref_tree.py --no-manifest --out $OUT/c5_ref_hash.json || exit 1
        timeout -k 10 300 python -u tools/hash_gpu_tree.py --out $OUT/c5_gpu_hash.json || exit 1 ;;
    tests)
        timeout -k 10 900 python -u -m pytest tests/test_group.py tests/test_gpu_parity.py tests/test_gpu_cost_order.py \
            -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; } ;;
    alltests)
        timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
            > $OUT/pytest_all.log 2>&1 || { tail -30 $OUT/pytest_all.log; exit 1; } ;;
    c3)
        timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1 ;;
    c5)
        timeout -k 10 400 python -u bench.py --config c5 --steps 10 --no-cpu-baseline \
            > $OUT/bench_c5.json 2> $OUT/bench_c5.err || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
    esac
    echo "step $step ok"
done
