#!/bin/bash
# Build libtuplewise variants that differ only in count.hip compile-time knobs (CPU side):
#   tools/variants/libtuplewise_<tag>.so   for tools/count_variants.py on the GPU box.
# Usage: build_count_variants.sh "tag:-DDEFINE ..." ...   (SRC=rankcount.hip to vary that file)
set -e
cd "$(dirname "$0")/.."
C=trade-offs-in-distributed-tuplewise-estimation-and-learning_amd/csrc
make -C $C >/dev/null
mkdir -p tools/variants
SRC=${SRC:-count.hip}
OTHERS=$(ls $C/*.o | grep -v "/${SRC%.hip}.o$")
build() {  # tag, defines...
  local tag=$1; shift
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off "$@" \
    -c $C/$SRC -o /tmp/count_$tag.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/variants/libtuplewise_$tag.so \
    /tmp/count_$tag.o $OTHERS
  echo built $tag
}
for v in "$@"; do
  tag=${v%%:*}; defs=${v#*:}
  build $tag $defs &
done
wait
