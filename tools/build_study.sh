#!/bin/bash
# Builds a study variant of the engine library: tools/libjlcrc_<name>.so with
# extra compile flags (e.g. -DJL_LS_NOFOLD=1), in its own object tree.  Used with
# JLCRC_STUDY_LIB=tools/libjlcrc_<name>.so for A/B timings; never the product.
# Usage: bash tools/build_study.sh <name> [flags...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s -j8 -C jleveldb_amd/csrc STUDY=${STUDY:-1} BUILD=_build_$name OUT=../../tools/libjlcrc_$name.so EXTRA="$*"
