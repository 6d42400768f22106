#!/bin/bash
# Rebuilds the full source of a measured-and-rejected kernel variant from its patch under
# tools/probes/history/ (DESIGN.md §6 cites each one).  A patch's first line names its base: a
# product file at the commit where the variant was measured ("# base: <commit>:<path>", needs the
# git history, i.e. run it in the repository, not on the GPU box), or another history patch
# ("# base: patch:<name>.patch").
#   bash tools/probes/restore_variant.sh persistent_r02_pq2_fused [out.hip]
#   then build it like an ablation: hipcc ... -DFUSED_SRC='"<dir>/fused.hip"' window_probe.hip
set -euo pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
restore() {  # restore <name> <out>
  local p="$HERE/history/$1.patch"
  local base
  base=$(head -1 "$p" | sed 's/^# base: //')
  local tmp
  tmp=$(mktemp)
  if [[ "$base" == patch:* ]]; then
    restore "$(basename "${base#patch:}" .patch)" "$tmp"
  else
    git -C "$HERE" show "$base" > "$tmp"
  fi
  tail -n +2 "$p" | patch -s -o "$2" "$tmp"
  rm -f "$tmp"
}
name=$1
out=${2:-$HERE/build/$name/$(echo "$name" | sed -E 's/.*_(fused|wide)$/\1/').hip}
mkdir -p "$(dirname "$out")"
restore "$name" "$out"
echo "$out"
