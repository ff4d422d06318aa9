#!/bin/bash
# Build a copy of the package with extra hipcc flags for an A/B run (on the CPU host):
#   scripts/ab_variant.sh NAME "-DFOO=1"   ->  ab/NAME/{dash_amd,bench.py}
# then on the GPU box:  python ab/NAME/bench.py ...   (imports ab/NAME/dash_amd)
set -e
NAME=${1:?name}
FLAGS=${2:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
DST="$ROOT/ab/$NAME"
mkdir -p "$DST"
rm -rf "$DST/dash_amd" && cp -r "$ROOT/dash_amd" "$DST/"
find "$DST/dash_amd" -name "*.so" -delete
rm -rf "$DST/dash_amd/__pycache__"
cp "$ROOT/bench.py" "$DST/"
cd "$DST" && DASH_BUILD_DIR="$ROOT/build/ab_$NAME" DASH_HIP_FLAGS="$FLAGS" python -m dash_amd._build
