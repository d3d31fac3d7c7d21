#!/bin/bash
# Build an A/B variant of libvmatting.so from the current sources with one sed edit applied to one source file:
#   bash scripts/build_variant.sh <out.so> <csrc file> '<sed expression>'
# (objects of the other sources come from video-matting_amd/build; the variant goes to ab/, loaded via VM_LIB_PATH)
set -e
cd "$(dirname "$0")/../video-matting_amd"
make -s -j8 >/dev/null
OUT=$1; SRC=$2; EXPR=$3
TMP=$(mktemp -d)
sed "$EXPR" "csrc/$SRC" > "$TMP/$SRC"
cmp -s "csrc/$SRC" "$TMP/$SRC" && { echo "sed expression changed nothing"; exit 1; }
EXTRA=""; [ "$SRC" = "augment.hip" ] || [ "$SRC" = "loader.hip" ] && EXTRA="-ffp-contract=off"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wall -Wno-unused-function \
  -munsafe-fp-atomics $EXTRA -c "$TMP/$SRC" -o "$TMP/$SRC.o"
OBJS=$(ls build/*.o | grep -v "build/$SRC.o")
mkdir -p ../ab
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "../ab/$OUT" $OBJS "$TMP/$SRC.o"
rm -rf "$TMP"
echo "built ab/$OUT"
