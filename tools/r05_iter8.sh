#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
VARIANTS="base new2 new3 mfma16 base new2 new3 mfma16" bash tools/r05_iter3.sh
