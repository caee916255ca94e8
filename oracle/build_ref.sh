#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY — builds the reference's own CPU render path into oracle/_ref/.
#
# The reference (Alabuta/RaytracingInOneWeekend) is an MSVC/vcpkg project: g++ 11 rejects
# its sources as shipped. This recipe compiles them with three mechanical portability
# patches that touch no arithmetic:
#   1. `typename std::enable_if_t<...>* = 0>` -> `= nullptr>` (src/math.hxx x20,
#      src/raytracer.hxx:52): GCC rejects an int->void* default template argument;
#   2. `-include cfloat`: FLT_MIN is used at src/math.hxx:223 without its header;
#   3. src/raytracer.hxx:196 `static_assert(std::false_type{}, ...)` in a discarded
#      `if constexpr` branch -> the dependent `static_assert(sizeof(type) == 0, ...)`.
# The patched copy lives in a temporary directory OUTSIDE the repository and is deleted
# afterwards; only the binaries land in oracle/_ref/ (git-ignored). Reference sources are
# never copied into the repo. Nothing else (no cmake, no glm, no CUDA, no stand-in
# headers) is involved: the harness (oracle/ref_harness.cpp, our own code) #includes the
# reference's src/main.cxx and re-drives its dead CPU path (src/main.cxx:120-215).
#
# Outputs:
#   oracle/_ref/ref_harness_mt   — verbatim std::mt19937 engines (stream-exact renders)
#   oracle/_ref/ref_harness_pcg  — std::mt19937 replaced by a per-sample PCG32 engine
#                                  through a macro in the harness (no source edit)
set -euo pipefail
REF=${RT_REFERENCE:-/root/reference}
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
OUT="$HERE/_ref"
if [ ! -f "$REF/src/main.cxx" ]; then
    echo "build_ref: reference not present at $REF — skipping (prebuilt oracle/_ref used if any)" >&2
    exit 0
fi
mkdir -p "$OUT"
SCRATCH="$(mktemp -d /tmp/rt_ref_build.XXXXXX)"
trap 'rm -rf "$SCRATCH"' EXIT
cp -r "$REF/src" "$SCRATCH/src"
chmod -R u+w "$SCRATCH/src"
# patch 1
sed -i 's/\* = 0>/* = nullptr>/g' "$SCRATCH/src/math.hxx" "$SCRATCH/src/raytracer.hxx"
# patch 3
sed -i 's/else static_assert(std::false_type{}, "unsupported material type");/else static_assert(sizeof(type) == 0, "unsupported material type");/' \
    "$SCRATCH/src/raytracer.hxx"
grep -q 'sizeof(type) == 0' "$SCRATCH/src/raytracer.hxx" || { echo "build_ref: patch 3 did not apply" >&2; exit 1; }
# Same flags as the reference's Release build for the arithmetic that matters:
# -O3, no fast-math, baseline x86-64 (no FMA contraction possible).
CXX=${CXX:-g++}
FLAGS="-std=c++20 -O3 -DNDEBUG -include cfloat -I$SCRATCH/src -pthread"
$CXX $FLAGS -o "$OUT/ref_harness_mt.tmp" "$HERE/ref_harness.cpp"
$CXX $FLAGS -DRT_REF_ENGINE_PCG -o "$OUT/ref_harness_pcg.tmp" "$HERE/ref_harness.cpp"
mv "$OUT/ref_harness_mt.tmp" "$OUT/ref_harness_mt"
mv "$OUT/ref_harness_pcg.tmp" "$OUT/ref_harness_pcg"
echo "build_ref: built $OUT/ref_harness_mt $OUT/ref_harness_pcg"
