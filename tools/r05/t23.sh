#!/bin/bash
# Round 5: t22 (load rate vs rows per instruction) then t21 (the reduction's nt B with the ring, traffic)
bash tools/r05/t22.sh && bash tools/r05/t21.sh
