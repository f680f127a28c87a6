#!/bin/bash
# Round 5: k_embed_bwd2 (quad-split softmax, e1_w in LDS, two-ahead loads) against k_embed_bwd, and the inner update's
# entropy metrics in the update's launch (toued_agent_step_entropy): parity, timing, C2
E=$(pwd)/to-ued_amd/exp/libtoued_
B="python tools/bench_embed.py --blocks 768,384,1024,1536,2048"
C="python bench.py --steps 5 --warmup 2 --no_cpu_baseline --workloads none"
bash tools/gpu_steps.sh r05t35 \
  "par:400:python -u -m pytest tests/test_gpu_meta.py tests/test_gpu_sampler.py tests/test_gpu_api.py tests/test_gpu_curve.py -q -x --timeout 200 --timeout-method thread" \
  "emb:300:TOUED_LIB=${E}EMBED_V_1.so $B --save gpurun_out/r05t35/g1.pt && $B --save gpurun_out/r05t35/g2.pt && TOUED_LIB=${E}EMBED_WPE_4.so $B && python -c \"import torch; a=torch.load('gpurun_out/r05t35/g1.pt'); b=torch.load('gpurun_out/r05t35/g2.pt'); print('v2 vs v1 rel', float((a-b).norm()/a.norm()), 'max', float((a-b).abs().max()))\"" \
  "c2:400:TOUED_LIB=${E}EMBED_V_1.so TOUED_STEP_ENTROPY=0 $C && $C && TOUED_LIB=${E}EMBED_V_1.so TOUED_STEP_ENTROPY=0 $C && $C"
