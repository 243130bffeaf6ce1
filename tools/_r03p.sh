bash tools/gpu_profile.sh r03p && timeout -k 10 300 python3 tools/bench_bert_gemm.py > gpurun_out/r03p_bert_gemm.txt 2>&1; cat gpurun_out/r03p_bert_gemm.txt
