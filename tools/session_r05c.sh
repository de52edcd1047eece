set -u
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_launch_variants.py tests/test_gpu_parity_configs.py -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests rc=$?"; exit 1; }
echo tests ok
for r in 1 2 3; do
  for L in default nosort; do
    if [ $L = default ]; then unset VR_LIBRARY; else export VR_LIBRARY=$PWD/abx/libnosort.so; fi
    timeout -k 10 200 python bench.py --config c1 --steps 20 --warmup 2 --no-pmc --no-cpu-baseline --no-drop-in > $O/c1_${L}_$r.json 2> $O/c1_${L}_$r.err || { echo "c1 rc=$?"; exit 1; }
  done
done
unset VR_LIBRARY
echo c1 done
for r in 1 2; do for n in quantized full; do P=""; [ $r = 2 ] && P="--no-pmc"
  timeout -k 10 400 python bench.py --config c5 --nodes $n --steps 2 --warmup 1 --no-cpu-baseline --no-drop-in $P > $O/c5_${n}_$r.json 2> $O/c5_${n}_$r.err || { echo "c5 rc=$?"; exit 1; }
done; done
echo c5 done
