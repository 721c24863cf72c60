#!/bin/bash
# CPU AddressSanitizer build of the C-ABI host code (host side only: -fsanitize right after
# -Xarch_host; device code compiles as usual) + the driver -> ds-gan_amd/build/asan/asan_driver.
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/ds-gan_amd/csrc
O=$R/ds-gan_amd/build/asan
mkdir -p "$O"
FL="-O1 -g -std=c++17 --offload-arch=gfx950 -I$C -Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer"
objs=""
pids=""
for s in "$C/capi.cpp" "$C/thin3.hip" "$C/tconv.hip" "$C/skinny.hip" "$C/pwsmall.hip" \
         "$R/tools/asan/asan_stubs.cpp" "$R/tools/asan/asan_driver.cpp"; do
  o="$O/$(basename "$s").o"
  if [ ! -f "$o" ] || [ "$s" -nt "$o" ] || [ "$C/common.h" -nt "$o" ]; then
    /opt/rocm/bin/hipcc $FL -c "$s" -o "$o" &
    pids="$pids $!"
  fi
  objs="$objs $o"
done
for p in $pids; do wait "$p"; done   # (set -e: a failed compile stops the build)
/opt/rocm/bin/hipcc -Xarch_host -fsanitize=address $objs -o "$O/asan_driver"
echo "$O/asan_driver"
