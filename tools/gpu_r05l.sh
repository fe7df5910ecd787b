#!/bin/bash
# r05 session L: 87-state tiled RTS gains; k_cr_back_all per-workgroup timeline; linearize prefetch (pose row + observations before the table barrier) A/B vs committed
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
B=$PWD/acinoset_amd/csrc/build
step() { local n=$1 l=$2; shift 2; local t0=$(date +%s); timeout -k 10 $l "$@" > $OUT/$n.log 2>&1; local rc=$?;
  echo "[$n] rc=$rc $(( $(date +%s)-t0 ))s"; tail -n ${TAILN:-4} $OUT/$n.log; case $rc in 0|1) ;; *) echo fatal; exit $rc;; esac; }
TAILN=8 step pytest_ekf_r05l 600 python -u -m pytest tests/test_gpu_ekf.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "gains or default"
step ekfdef 300 rocprofv3 --kernel-trace --stats -d $OUT/ekfdef -o run -- python3 tools/time_ekf_leg.py default fd
find $OUT/ekfdef -name '*kernel_stats.csv' -exec cp {} $OUT/ekfdef_stats.csv \; ; head -12 $OUT/ekfdef_stats.csv | cut -c1-150; rm -rf $OUT/ekfdef
step pytest_fte_r05l 600 python -u -m pytest tests/test_gpu_fte.py tests/test_gpu_fte_cfg2.py tests/test_gpu_fullsize.py -k "fte or FTE or cfg" -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for v in main base; do
  if [ $v = main ]; then unset ACINOSET_HIP_LIB; else export ACINOSET_HIP_LIB=$B/libvar_base.so; fi
  step tr10k_$v 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr10k_$v -o run -- python3 tools/prof_fte.py --frames 10000 --reps 2
  python tools/fte_iter_sequence.py $OUT/tr10k_$v > $OUT/seq10k_$v.log 2>&1; grep -E "linearize|assemble|back_all|kernels" $OUT/seq10k_$v.log | head -5
  step tr1k_$v 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr1k_$v -o run -- python3 tools/prof_fte.py --frames 1000 --reps 3
  python tools/fte_iter_sequence.py $OUT/tr1k_$v > $OUT/seq1k_$v.log 2>&1; grep -E "linearize|assemble|back_all|kernels" $OUT/seq1k_$v.log | head -5
  rm -rf $OUT/tr10k_$v $OUT/tr1k_$v
done
unset ACINOSET_HIP_LIB
step backtr10k 300 python tools/prof_back_all.py 10000
TAILN=20 step backtr1k 300 python tools/prof_back_all.py 1000
cat $OUT/backtr10k.log
echo done
