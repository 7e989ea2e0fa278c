set -o pipefail
mkdir -p gpurun_out/s4
for cfg in C2B4 C2S8 x1,32,8192,128,1 x8,16,2048,128,1 x1,32,4096,64,1; do
  timeout -k 10 150 python -u tools/ab_fwd.py MFA_FWD_STREAM=0,1 --cfg $cfg --rounds 6 > gpurun_out/s4/ab_$cfg.txt 2>&1 || { tail -5 gpurun_out/s4/ab_$cfg.txt; exit 1; }
  grep cfg gpurun_out/s4/ab_$cfg.txt
done
