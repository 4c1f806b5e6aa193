# build an A/B variant of the library from an alternative dynamics source:
#   bash tools/build_variant.sh <name> [dynamics.hip source (default: the tree's)] [extra hipcc flags...]
# -> ti5_isaacgym_amd/_lib/var/<name>.so (the tree's source is restored afterwards)
set -e
name=$1; shift
src=${1:-}; [ $# -gt 0 ] && shift
D=ti5_isaacgym_amd/csrc/t1env_dynamics.hip
if [ -n "$src" ] && [ "$src" != "-" ]; then cp $D /tmp/_bv_keep.hip; cp $src $D; fi
mkdir -p ti5_isaacgym_amd/_lib/var/$name.d
python -m ti5_isaacgym_amd.build --out=$PWD/ti5_isaacgym_amd/_lib/var/$name.d/lib.so "$@" > /dev/null || { [ -n "$src" ] && [ "$src" != "-" ] && cp /tmp/_bv_keep.hip $D; exit 1; }
mv ti5_isaacgym_amd/_lib/var/$name.d/lib.so ti5_isaacgym_amd/_lib/var/$name.so; rm -rf ti5_isaacgym_amd/_lib/var/$name.d
if [ -n "$src" ] && [ "$src" != "-" ]; then cp /tmp/_bv_keep.hip $D; fi
echo ti5_isaacgym_amd/_lib/var/$name.so
