#!/bin/bash
# Round-4 GPU call: the whole GPU suite + smoke after the phased-dgrad workspace fix.
bash tools/round_final.sh
