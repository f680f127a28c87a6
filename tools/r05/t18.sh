#!/bin/bash
# Round 5: the load path per CU vs loads in flight and cache policy (tools/load_probe.hip)
mkdir -p gpurun_out/r05t18
hipcc -O3 --offload-arch=gfx950 tools/load_probe.hip -o /tmp/load_probe && timeout -k 10 120 /tmp/load_probe > gpurun_out/r05t18/probe.log 2>&1; cat gpurun_out/r05t18/probe.log
