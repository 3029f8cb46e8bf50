#!/bin/bash
#-------------------------------------------------------------
# Two-step decision-tree data generation (reference scripts/datagen/genRandData4DecisionTree.sh).
#   genRandData4DecisionTree.sh <outdir> [records] [scale feats] [cat feats] [classes] [distinct] [sparsity] [fmt]
#-------------------------------------------------------------
set -e
OUT=${1:-dt_data}; N=${2:-1000}; NS=${3:-5}; NC=${4:-3}; K=${5:-3}; D=${6:-5}; SP=${7:-1.0}; FMT=${8:-csv}
HERE=$(cd "$(dirname "$0")" && pwd)
mkdir -p "$OUT"
python -m systemml_amd -f "$HERE/genRandData4DecisionTree1.dml" -nvargs XCat="$OUT/XCat" Y="$OUT/Y" \
  num_records=$N num_cat=$NC num_class=$K num_distinct=$D sp=$SP
cols=$(seq -s, 1 $NC)
echo "{\"ids\": true, \"recode\": [$cols], \"dummycode\": [$cols]}" > "$OUT/tspec.json"
python -m systemml_amd -f "$HERE/genRandData4DecisionTree2.dml" -nvargs XCat="$OUT/XCat" X="$OUT/X" \
  num_records=$N num_scale=$NS sp=$SP fmt=$FMT tSpec="$OUT/tspec.json" tPath="$OUT/tmeta"
