#!/bin/bash
# queues A/B on the headline loop, then the --gpus 8 rehearsal with the tile lines on one GPU.
set -o pipefail
tag=$1
bash tools/gpu_runs/r06/queues_ab.sh $tag || exit 1
bash tools/gpu_rehearse8_tiles.sh ${tag}_r8 || exit 1
