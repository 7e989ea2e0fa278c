# AGPR-owning forward: parity, stamps, then one-process A/B against the shipped kernels.
set -o pipefail
O=gpurun_out/${1:-aw}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_forward_aw_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 tools/diag/aw_stamps 16 8192 0 > $O/stamps_c3.txt 2>&1 || { cat $O/stamps_c3.txt; exit 1; }
cat $O/stamps_c3.txt
for cfg in ${CFGS:-C3 C2}; do
  timeout -k 10 150 python -u tools/ab_fwd.py MFA_FWD_AW=0,1 --cfg $cfg --rounds 6 > $O/ab_$cfg.txt 2>&1 || { tail -5 $O/ab_$cfg.txt; exit 1; }
  grep cfg $O/ab_$cfg.txt
done
