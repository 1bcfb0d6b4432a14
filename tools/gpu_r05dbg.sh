# round 5: why does tests/test_gpu_bench.py stall on the box? mtimes of the build inputs there, a
# dry-run make, then the test's bench command with its own timing
set -o pipefail
O=gpurun_out/r05dbg; mkdir -p $O
ls --full-time element-crush-gym_amd/csrc element-crush-gym_amd/build include > $O/mtimes.txt 2>&1
make -n -C element-crush-gym_amd > $O/make_n.txt 2>&1; echo "make -n lines: $(wc -l < $O/make_n.txt)"
( time timeout -k 10 60 make -s -C element-crush-gym_amd ) > $O/make.txt 2>&1; echo "make rc=$?"; tail -3 $O/make.txt
( time timeout -k 10 150 python3 -u bench.py --shape 9x9x6 --boards 65536 --steps 6 --warmup 3 --no-cpu-baseline --check-boards 384 ) > $O/bench.txt 2>&1
echo "bench rc=$?"; tail -c 400 $O/bench.txt
