#!/bin/bash
# Builds and runs the golden generator against the survey's CPU build of the reference
# (/tmp/ocvbuild, configured from a patched copy of /root/reference).
# Test infrastructure only: runs in the build container, never on the GPU box.
set -euo pipefail
REF=${REF:-/root/reference}
OCV=${OCV:-/tmp/ocvbuild}
OUT=${1:-/tmp/golden_raw}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
INC="-I$OCV"
for m in core imgproc calib3d features2d flann stitching octvr imgcodecs videoio highgui ml objdetect; do
  INC="$INC -I$REF/modules/$m/include"
done
g++ -std=c++11 -O1 -w $INC "$HERE/gen_golden.cpp" -o /tmp/gen_golden \
  -L"$OCV/lib" -lopencv_octvr -lopencv_stitching -lopencv_calib3d -lopencv_features2d \
  -lopencv_imgproc -lopencv_core -Wl,-rpath,"$OCV/lib"
/tmp/gen_golden "$OUT"
python3 "$HERE/pack_golden.py" "$OUT" "$HERE/../../tests/golden"
