#!/bin/bash
# Round 5: the store / load path per CU at 8 .. 256 workgroups (tools/store_probe.hip)
mkdir -p gpurun_out/r05t15
hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o /tmp/store_probe && timeout -k 10 120 /tmp/store_probe | tee gpurun_out/r05t15/probe.log
