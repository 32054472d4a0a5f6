# A/B of element-wise launch variants (upmem--openfhe_amd/lib/variants) with tools/eltwise_bw.py
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/elt
for v in ${ELT_VARIANTS:-main}; do
  if [ $v = main ]; then L=""; else L=upmem--openfhe_amd/lib/variants/libofhe_hip_$v.so; fi
  EXP_LIB=$L timeout -k 10 120 python3 tools/eltwise_bw.py > gpurun_out/elt/$v.$RANDOM.json
  echo done $v
done
