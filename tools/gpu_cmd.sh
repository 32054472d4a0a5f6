EXP_CONFIGS=";OFHE_SPLIT4=1;OFHE_NO_SPQ=1;OFHE_SPLIT4=1,OFHE_NO_SPQ=1" timeout -k 10 300 python tools/exp_variants.py > gpurun_out/exp_var.txt 2>&1; cat gpurun_out/exp_var.txt
SKIP_BENCH=1 bash tools/gpu_round.sh
