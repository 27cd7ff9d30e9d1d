#!/bin/bash
# face tests + probe (tile kernel on colour items), then the XC tests and 2/4-rank detached benches
set -o pipefail
bash scripts/face_wave_check.sh tile1 || exit 1
bash scripts/xc_mp_check.sh || exit 1
