"""CPU: the short-latency f64 helpers of acinoset_amd/csrc/fastmath.hpp (log1p_pos, the
rcp/rsq wrappers), built with g++ from the same header the kernels include and checked
against libm. On the device rcp_nr / rsq_nr refine the hardware estimates by two Newton
steps; the GPU parity tests cover that path end to end."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

SRC = r'''
#include <cstdio>
#include <random>
#include "fastmath.hpp"
int main() {
  std::mt19937_64 g(7);
  double worst = 0.0;
  for (int i = 0; i < 400000; ++i) {
    const double e = std::uniform_real_distribution<double>(-70.0, 40.0)(g);
    double t = std::ldexp(std::uniform_real_distribution<double>(1.0, 2.0)(g), (int)e);
    if (i < 64) t = i * 0.125;
    const double a = log1p_pos(t), b = std::log1p(t);
    const double ulp = b == 0.0 ? (a == 0.0 ? 0.0 : 1e9) : std::fabs(a - b) / (std::nextafter(b, INFINITY) - b);
    if (ulp > worst) worst = ulp;
  }
  double worst_atan = 0.0;
  for (int i = 0; i < 400000; ++i) {
    const double e = std::uniform_real_distribution<double>(-40.0, 40.0)(g);
    double x = std::ldexp(std::uniform_real_distribution<double>(1.0, 2.0)(g), (int)e);
    if (i < 64) x = i * 0.0625;
    const double a = atan_pos(x), b = std::atan(x);
    const double ulp = b == 0.0 ? (a == 0.0 ? 0.0 : 1e9) : std::fabs(a - b) / (std::nextafter(b, INFINITY) - b);
    if (ulp > worst_atan) worst_atan = ulp;
  }
  printf("%.3f %.3f\n", worst, worst_atan);
  return 0;
}
'''


@pytest.mark.skipif(shutil.which('g++') is None, reason='g++ not available')
def test_log1p_and_atan_within_ulps(tmp_path):
    src = tmp_path / 'fm.cpp'
    src.write_text(SRC)
    exe = tmp_path / 'fm'
    subprocess.run(['g++', '-O2', '-std=c++17', '-I', os.path.join(REPO, 'acinoset_amd', 'csrc'), str(src), '-o',
                    str(exe)], check=True)
    worst, worst_atan = map(float, subprocess.run([str(exe)], capture_output=True, text=True,
                                                  check=True).stdout.split())
    assert worst <= 1.0, worst
    assert worst_atan <= 4.0, worst_atan  # the pi/4 branch near tan(pi/8) loses ~2 bits
