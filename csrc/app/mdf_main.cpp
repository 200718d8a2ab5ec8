// `mdf`: the reference MDF program (MDF_kernel.cu) — 2D 5-point heat/Jacobi, Dirichlet edges 100,
// interior 0 — with the same stdin dialogue, on the mdfx engine.
#include "cli_common.hpp"
int main(int argc, char** argv) { return mdfx::run_cli(argc, argv, "jacobi5", "mdf"); }
