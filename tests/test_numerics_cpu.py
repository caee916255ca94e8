"""Exhaustive checks of the exact rewrites the kernel relies on (rt_kernel.hip):
with a correctly rounded sqrt (IEEE on x86 and the hipcc sequence on gfx950),
  sqrtf(n) > 1   <=>  n > 0x1.000002p+0f   (random_in_unit_sphere, raytracer.hxx:41)
  sqrtf(n) > 0   <=>  n > 0                (length(refracted) > 0, raytracer.hxx:180)
for every non-negative float n (all 2^31 bit patterns, NaN included)."""
import subprocess

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
int main(void) {
  unsigned long long bad = 0;
  for (uint64_t b = 0; b <= 0x7fffffffu; ++b) {
    uint32_t u = (uint32_t)b; float n; memcpy(&n, &u, 4);
    float r = sqrtf(n);
    bad += (r > 1.f) != (n > 0x1.000002p+0f);
    bad += (r > 0.f) != (n > 0.f);
  }
  printf("%llu\n", bad);
  return bad != 0;
}
"""


def test_sqrt_comparison_rewrites_exhaustive(tmp_path):
    c = tmp_path / "eq.c"
    c.write_text(SRC)
    exe = tmp_path / "eq"
    subprocess.run(["gcc", "-O2", "-fno-fast-math", str(c), "-o", str(exe), "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip() == "0", r.stdout
