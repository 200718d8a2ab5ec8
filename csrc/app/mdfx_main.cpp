// `mdfx`: the general front end (2D/3D stencils, fp32/fp64, GPUs, transports, benchmarks).
// Without size/step flags it runs the reference MDF dialogue.
#include <cstring>

#include "cli_common.hpp"
int main(int argc, char** argv) {
  // bare `mdfx` behaves like the reference MDF program; with flags the default stencil is 3D 7-pt
  bool flags = false;
  for (int i = 1; i < argc; ++i)
    if (std::strncmp(argv[i], "--", 2) == 0 && std::strcmp(argv[i], "--print") != 0 &&
        std::strcmp(argv[i], "--compat") != 0)
      flags = true;
  return mdfx::run_cli(argc, argv, flags ? "heat7" : "jacobi5", "mdfx");
}
