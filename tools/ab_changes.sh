# dg_join2_changes A/B (config 2, synchronous calls): every libdeltagpu*.so in the tree.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
for l in $(cd delta_crdt_ex_amd && ls libdeltagpu*.so | grep -v stamps); do
  echo -n "$l: "; DG_LIB_PATH=$PWD/delta_crdt_ex_amd/$l timeout -k 10 200 python -u tools/prof_changes.py 2>&1 | tr '\n' ' ' || exit 1; echo
done
done
