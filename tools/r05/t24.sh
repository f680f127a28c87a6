#!/bin/bash
# Round 5: a CU's load rate vs rows (cache lines) per wave instruction (tools/load_probe2.hip)
mkdir -p gpurun_out/r05t24
hipcc -O3 --offload-arch=gfx950 tools/load_probe2.hip -o /tmp/load_probe2 && timeout -k 10 120 /tmp/load_probe2 > gpurun_out/r05t24/probe.log 2>&1; cat gpurun_out/r05t24/probe.log
