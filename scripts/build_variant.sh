#!/bin/bash
# Build a variant of libmafrix_rt.so into build_variants/NAME.so with extra compiler flags, for
# scripts/ab_variants.py. Usage: scripts/build_variant.sh NAME [-DFOO=1 ...] [--src DIR]
set -e
R=$(cd $(dirname $0)/.. && pwd)
NAME=$1; shift
SRC=$R/mafrixraytracing_amd/csrc
if [ "$1" == "--src" ]; then SRC=$2; shift 2; fi
OUT=${MFX_VARIANT_DIR:-$R/build_variants}  # (build_ab/: A/B candidates, scripts/ab_variants.py MFX_AB_DIR)
mkdir -p $OUT
cd $SRC
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wall -Wno-unused-result \
  -I$R/include "$@" -shared -o $OUT/$NAME.so $(ls *.cpp *.hip) -ldl
