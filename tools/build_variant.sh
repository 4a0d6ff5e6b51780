# Builds a variant of the library into variants/<name>.so (pushed to the GPU box; not committed) from a copy of the sources with extra
# compile flags (A/B experiments, tools/ab.sh).  usage: bash tools/build_variant.sh NAME "-DFOO=1"
set -e
ROOT=$(cd $(dirname $0)/.. && pwd)
D=/tmp/bgvar_$1/x
rm -rf /tmp/bgvar_$1; mkdir -p $D/csrc /tmp/bgvar_$1/include
cp $ROOT/biogarden_amd/csrc/*.hip $ROOT/biogarden_amd/csrc/*.h $ROOT/biogarden_amd/csrc/*.cpp $ROOT/biogarden_amd/csrc/*.inc $ROOT/biogarden_amd/csrc/Makefile $D/csrc/
cp $ROOT/include/*.h /tmp/bgvar_$1/include/
mkdir -p $ROOT/variants
make -s -C $D/csrc -j8 OUT=$ROOT/variants/$1.so FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -I../../include -Wall $2"
echo "built variants/$1.so ($2)"
