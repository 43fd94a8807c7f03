mkdir -p gpurun_out/r06 && timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "heavy_first or pixel" > gpurun_out/r06/hf_tests.log 2>&1 || exit 1
A=octreeraytracer_amd/lib/libort_analysis.so
run() { name=$1; shift; timeout -k 10 240 python tools/ab_stream.py $A@pixel_heavy_first=0 $A@pixel_heavy_first=1 "$@" > gpurun_out/r06/ab_hf_$name.log 2>&1 || exit 1; }
run ref_default --config ref_default
run ref_stats114 --config ref_stats114
run c2d4 --config c2 --max-depth 4
run c2s4d8 --config c2 --samples 4 --max-depth 8
run mid30k --config c2 --spheres 30000 --tree-depth 7 --samples 4 --max-depth 8
run mid30k_s2 --config c2 --spheres 30000 --tree-depth 7 --samples 2 --max-depth 4
