// smp_node::normalizeTrajectory of the C++ shim (include/smp_birrt_star.hpp) on trajectories read from stdin:
//   dim n  then n rows of dim values, then the dim normalized distances; repeated until EOF.
// Prints per case "rows m" and the rows with %.17g (or "untouched" when the reference leaves the output as is).
#include <cstdio>
#include <vector>

#include "smp_birrt_star.hpp"

int main() {
  int dim, n;
  while (std::scanf("%d %d", &dim, &n) == 2) {
    std::vector<std::vector<double> > raw(n, std::vector<double>(dim));
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < dim; ++j)
        if (std::scanf("%lf", &raw[i][j]) != 1) return 2;
    std::vector<double> np(dim);
    for (int j = 0; j < dim; ++j)
      if (std::scanf("%lf", &np[j]) != 1) return 2;
    std::vector<std::vector<double> > out(1, std::vector<double>(1, 42.0));  // sentinel: untouched?
    smp_node::normalizeTrajectory(raw, out, np);
    if (out.size() == 1 && out[0].size() == 1 && out[0][0] == 42.0) {
      std::printf("untouched\n");
      continue;
    }
    std::printf("rows %zu\n", out.size());
    for (size_t i = 0; i < out.size(); ++i) {
      for (size_t j = 0; j < out[i].size(); ++j) std::printf("%s%.17g", j ? " " : "", out[i][j]);
      std::printf("\n");
    }
  }
  return 0;
}
