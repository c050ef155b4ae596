#!/bin/bash
# smoke + full bench line, then the rocprofv3 trace and PMC passes of the headline (tools/measure.sh).
set -o pipefail
tag=$1
bash tools/gpu_runs/r06/bench_full.sh $tag || exit 1
bash tools/measure.sh $tag trace pmc || exit 1
