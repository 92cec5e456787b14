#!/bin/bash
# Round-4 GPU call: kernel breakdown of one eager generator step and one critic step at the final build.
mkdir -p gpurun_out
timeout -k 10 600 bash tools/phase_trace.sh r04cc > gpurun_out/r04cc_phase.log 2>&1
