// `life`: the reference Game-of-Life program (kernel.cu) — Moore-8 B3/S23, dead frame, glibc rand()
// Bernoulli(0.15) initial board — with the same stdin dialogue, on the mdfx engine.
#include "cli_common.hpp"
int main(int argc, char** argv) { return mdfx::run_cli(argc, argv, "life", "life"); }
