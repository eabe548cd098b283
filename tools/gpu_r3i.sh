#!/bin/bash
set -o pipefail
bash tools/pmc_ops.sh c1 conv1c3_fwd conv1c3_wgrad
