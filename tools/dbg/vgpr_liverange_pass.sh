# Round 6: the lane interference of DESIGN.md §4 traced to LLVM's SIOptimizeVGPRLiveRange pass.
# Rebuilds the pre-fix tree (commit ca93999, the library that failed) three ways -- as it was built
# then, without stack-slot sharing, and without SIOptimizeVGPRLiveRange -- and runs the failing
# rollouts (tools/dbg/lanes_k.py 10x8x9) and the frame-rollout regression test on each.
# CPU part (here):  bash tools/dbg/vgpr_liverange_pass.sh build     (~15 min, writes dbg_libs/)
# GPU part:         gpurun -- 'bash tools/dbg/vgpr_liverange_pass.sh run'
set -o pipefail
case "$1" in
build)
  rm -rf /tmp/pre && mkdir -p /tmp/pre dbg_libs
  git archive ca93999 element-crush-gym_amd/csrc include | tar -x -C /tmp/pre
  git show ca93999:element-crush-gym_amd/Makefile > /tmp/pre/element-crush-gym_amd/Makefile
  ( cd /tmp/pre/element-crush-gym_amd &&
    make -j8 variant NAME=base &&
    make -j8 variant NAME=nossc XFLAGS='-mllvm -disable-ssc' &&
    make -j8 variant NAME=novlr XFLAGS='-mllvm -amdgpu-opt-vgpr-liverange=false' ) || exit 1
  cp /tmp/pre/element-crush-gym_amd/build/libm3_{base,nossc,novlr}.so dbg_libs/ ;;
run)
  O=gpurun_out/vlr; mkdir -p $O
  for L in base nossc novlr; do
    M3_LIB=$PWD/dbg_libs/libm3_$L.so timeout -k 10 300 python3 -u tools/dbg/lanes_k.py 10x8x9 > $O/lanes_$L.log 2>&1 || exit 1
    echo "== $L"; grep "^k=" $O/lanes_$L.log
    M3_LIB=$PWD/dbg_libs/libm3_$L.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_shapes.py -k frame_rollouts_vs_oracle \
      -m gpu -v --timeout 300 --timeout-method thread > $O/frame_rollouts_$L.log 2>&1
    grep -E "PASSED|FAILED" $O/frame_rollouts_$L.log | sed 's/.*:://' | head -7
  done ;;
*) echo "usage: $0 build|run"; exit 2 ;;
esac
