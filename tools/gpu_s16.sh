#!/bin/bash
# PMC passes over the isolated 720p attention backward (delta + dK/dV + dQ with split tails).
bash tools/pmc_kernels.sh ${1:-s16}_attn_bwd attn_bwd 1
