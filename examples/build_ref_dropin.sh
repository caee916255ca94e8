#!/usr/bin/env bash
# The INTEGRATION.md swap applied to the REFERENCE's own main() and compiled against
# librt_mi355x.so — the reference-side binding a maintainer would add, built with the
# reference's real types (raytracer::data, primitives::sphere, material::types, math::u8vec3).
#
# In a scratch copy of /root/reference/src OUTSIDE the repository (deleted afterwards):
#   * the three portability patches of oracle/build_ref.sh (no arithmetic change);
#   * src/main.cxx: `#include "rt_render_impl.hpp"`; the scene construction of main.cxx:120-129
#     moved above the render call (main.cxx:112); `cuda_impl(app_data.width, app_data.height,
#     output)` (main.cxx:114) replaced by
#         rt::render_impl(raytracer_data, app_data.width, app_data.height, output,
#                         rt::settings{app_data.sampling_number, raytracer_data.bounces_number});
#     everything else (app::data, save_to_file("image_cuda.ppm"), the dead CPU loop) unchanged.
# Built with -D_DEBUG, the reference's debug frame size (main.cxx:25-27: 512x256, 16 spp), so the
# test can compare its PPM with the reference's own render of that frame.
# Output: examples/_ref/ref_main_dropin (git-ignored; travels to the GPU box, rpath to the
# in-tree library). Never copies reference sources into the repository.
set -euo pipefail
REF=${RT_REFERENCE:-/root/reference}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(dirname "$HERE")"
OUT="$HERE/_ref"
if [ ! -f "$REF/src/main.cxx" ]; then
    echo "build_ref_dropin: reference not present at $REF — skipping" >&2
    exit 0
fi
mkdir -p "$OUT"
SCRATCH="$(mktemp -d /tmp/rt_ref_dropin.XXXXXX)"
trap 'rm -rf "$SCRATCH"' EXIT
cp -r "$REF/src" "$SCRATCH/src"
chmod -R u+w "$SCRATCH/src"
sed -i 's/\* = 0>/* = nullptr>/g' "$SCRATCH/src/math.hxx" "$SCRATCH/src/raytracer.hxx"
sed -i 's/else static_assert(std::false_type{}, "unsupported material type");/else static_assert(sizeof(type) == 0, "unsupported material type");/' \
    "$SCRATCH/src/raytracer.hxx"
python3 - "$SCRATCH/src/main.cxx" <<'EOF'
import sys
p = sys.argv[1]
L = open(p).read().split("\n")
def find(s, start=0):
    for i in range(start, len(L)):
        if s in L[i]:
            return i
    raise SystemExit(f"build_ref_dropin: anchor not found: {s!r}")
# the scene block: from the first material push_back after `return 0;` to the blank line before #if 0
ret = find("return 0;")
b0 = find("raytracer_data.materials.push_back(", ret)
b1 = find("#if 0", b0)
block = L[b0:b1]
del L[b0:b1]
call = find("cuda_impl(app_data.width, app_data.height, output);")
L[call] = L[call].replace("cuda_impl(app_data.width, app_data.height, output);",
                          "rt::render_impl(raytracer_data, app_data.width, app_data.height, output, "
                          "rt::settings{app_data.sampling_number, raytracer_data.bounces_number});")
data = find("raytracer::data raytracer_data;")
L[data + 1:data + 1] = block
inc = find('#include "camera.hxx"')
L.insert(inc + 1, '#include "rt_render_impl.hpp"')
open(p, "w").write("\n".join(L))
EOF
grep -q 'rt::render_impl(raytracer_data' "$SCRATCH/src/main.cxx" || { echo "build_ref_dropin: swap did not apply" >&2; exit 1; }
${CXX:-g++} -std=c++20 -O2 -D_DEBUG -include cfloat -I"$SCRATCH/src" -I"$REPO/include" -pthread \
    "$SCRATCH/src/main.cxx" -L"$REPO/raytracinginoneweekend_amd" -lrt_mi355x \
    -Wl,-rpath,'$ORIGIN/../../raytracinginoneweekend_amd' -o "$OUT/ref_main_dropin.tmp"
mv "$OUT/ref_main_dropin.tmp" "$OUT/ref_main_dropin"
echo "build_ref_dropin: built $OUT/ref_main_dropin"
