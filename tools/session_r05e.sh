set -u
O=gpurun_out/r05f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-drop-in > $O/c3_default.json 2> $O/c3_default.err || { echo "c3 rc=$?"; exit 1; }
VR_LIBRARY=$PWD/abx/librngdraw.so timeout -k 10 300 python bench.py --steps 3 --no-cpu-baseline --no-drop-in > $O/c3_rngdraw.json 2> $O/c3_rngdraw.err || { echo "rngid rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --no-pmc --no-cpu-baseline --no-drop-in > $O/c3_prof.json 2> $O/c3_prof.err || { echo "prof rc=$?"; exit 1; }
echo done
