#!/bin/bash
# profile_round.sh over the three single-GPU bench configurations:
#   <tag>    config #3 (256 x 1080p, the headline)
#   <tag>c2  config #2 (1 x 1080p)
#   <tag>c5  config #5 per-rank shard (64 x 4K, 5 octaves, rotated 128-D)
#   bash tools/profile_configs.sh <tag>
set -u
TAG=$1
cd "${GRAFT_REPO_ROOT:-/root/repo}"
bash tools/profile_round.sh ${TAG} || exit $?
bash tools/profile_round.sh ${TAG}c2 --batch 1 --no-exchange-probe || exit $?
bash tools/profile_round.sh ${TAG}c5 --batch 64 --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1 --no-exchange-probe || exit $?
echo CONFIGS_DONE
