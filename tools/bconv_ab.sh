# A/B of base-conversion variant builds (upmem--openfhe_amd/lib/variants) with tools/bconv_bw.py
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bconv
for v in ${BC_VARIANTS:-main}; do
  if [ $v = main ]; then L=""; else L=upmem--openfhe_amd/lib/variants/libofhe_hip_$v.so; fi
  EXP_LIB=$L timeout -k 10 120 python3 tools/bconv_bw.py | tee -a gpurun_out/bconv/results.jsonl
done
