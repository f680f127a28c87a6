#!/bin/bash
# Round 5: load layouts per CU (tools/store_probe.hip), then k_wgrad_h3's two-slab B ring (t16)
mkdir -p gpurun_out/r05t17
hipcc -O3 --offload-arch=gfx950 tools/store_probe.hip -o /tmp/store_probe && timeout -k 10 120 /tmp/store_probe > gpurun_out/r05t17/probe.log 2>&1 && cat gpurun_out/r05t17/probe.log && bash tools/r05/t16.sh
