"""The kernel reads an RGB8 texel back as b / 255 with q0 = b * RN(1/255) plus one fma correction
(csrc/vrt_render.hip unorm8_read) instead of an IEEE division. Exhaustive proof over the 256 byte
values that the sequence equals the correctly rounded quotient, run on the host's IEEE single
precision (glibc fmaf is correctly rounded, like v_fma_f32)."""
import os
import subprocess

SRC = r"""
#include <math.h>
#include <stdio.h>
#include <string.h>
int main(void) {
  const float y = 1.0f / 255.0f;
  int bad = 0;
  for (int b = 0; b < 256; b++) {
    const float a = (float)b, q0 = a * y, q = fmaf(fmaf(-255.0f, q0, a), y, q0), ref = a / 255.0f;
    unsigned u, v;
    memcpy(&u, &q, 4);
    memcpy(&v, &ref, 4);
    bad += u != v;
  }
  printf("%d\n", bad);
  return 0;
}
"""


def test_div255_sequence_is_exact(tmp_path):
    c = tmp_path / "div255.c"
    c.write_text(SRC)
    exe = tmp_path / "div255"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-o", str(exe), str(c),
                    "-lm"], check=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.strip() == "0"
