#!/bin/bash
# A/B of two source trees (e.g. an ABI change): tools/ab.py run from each tree with its own
# library, alternating trees, in one box session.   usage: gpu_ab_trees.sh <tree_a> <tree_b> [rounds]
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/abt; mkdir -p $O; export TMPDIR=/tmp
A=$1; B=$2; N=${3:-3}
for s in 0 1; do   # 0: the automatic group count
  for i in $(seq $N); do
    for T in $A $B; do
      (cd $T && SPGG_STREAMS=$s timeout -k 10 200 python tools/ab.py --config cfg3 --libs neighbor-aware-reinforcement-learning-fosters-cooperation-in-spatial-public-goods-games-_amd/libspgg_hip.so --steps 200 --rounds 2 2>&1 | grep -v amdgpu.ids | sed "s|^|streams $s $T: |") || exit 1
    done
  done
done
