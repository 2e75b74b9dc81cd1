#!/bin/bash
# Developer A/B builds: the working tree as lib/ab_B.so and the same tree with the listed
# files taken from a git revision as lib/ab_A.so.  usage: bash tools/build_ab.sh <rev> <file>...
set -e
REV=$1; shift
cd "$(dirname "$0")/.."
B=gripper-mujoco_amd/lib/ab_B.so; A=gripper-mujoco_amd/lib/ab_A.so
python -c "import sys; sys.path.insert(0,'gripper-mujoco_amd'); from gmx.build import build; build(out='$PWD/$B')"
SAVE=$(mktemp -d)
for f in "$@"; do mkdir -p $SAVE/$(dirname $f); cp $f $SAVE/$f; git show $REV:$f > $f; done
trap 'for f in "$@"; do cp $SAVE/$f $f; done' EXIT
python -c "import sys; sys.path.insert(0,'gripper-mujoco_amd'); from gmx.build import build; build(out='$PWD/$A')"
echo "built $A ($REV) and $B (working tree)"
