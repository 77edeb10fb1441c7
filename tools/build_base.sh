# Build libdeltagpu.so from an earlier commit's sources into delta_crdt_ex_amd/ab/ for an
# A/B against the working tree:  bash tools/build_base.sh <rev> [name]  (default name: base)
# Load it with DG_LIB_PATH=.../ab/libdeltagpu_<name>.so DG_LIB_ANY_DIGEST=1.
set -e
REV=${1:?rev}
NAME=${2:-base}
R=$(cd "$(dirname "$0")/.." && pwd)
W=$(mktemp -d /tmp/dgbase.XXXXXX)
git -C "$R" archive "$REV" delta_crdt_ex_amd/csrc delta_crdt_ex_amd/build.py delta_crdt_ex_amd/_abi.py include | tar -x -C "$W"
(cd "$W" && python -m delta_crdt_ex_amd.build > /dev/null)
mkdir -p "$R/delta_crdt_ex_amd/ab"
cp "$W/delta_crdt_ex_amd/libdeltagpu.so" "$R/delta_crdt_ex_amd/ab/libdeltagpu_$NAME.so"
rm -rf "$W"
echo "$R/delta_crdt_ex_amd/ab/libdeltagpu_$NAME.so"
