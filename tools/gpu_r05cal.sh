# round 5: FETCH_SIZE / WRITE_SIZE calibration for 16 / 4 / 1-byte-per-lane accesses (tools/calib)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05cal; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f --output-format csv -- ./tools/calib/fetch_calib > $O/f.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $O/w -o w --output-format csv -- ./tools/calib/fetch_calib > $O/w.log 2>&1
echo rc=$?
