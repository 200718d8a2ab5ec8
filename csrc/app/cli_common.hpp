// mdfx command-line front end shared by the `mdf`, `life` and `mdfx` executables.
//
// Reference parity: with no size/step flags the program runs the reference's stdin
// dialogue byte for byte (MDF_kernel.cu:105-112 / kernel.cu:152-159):
//     Enter desired number of generations:\n   (scanf %d)
//     Enter desired height of universe:\n      (scanf %d)
//     Enter desired width of universe:\n       (scanf %d)
// printed and read by rank 0 only, then broadcast (fixes D14). `--print` dumps the final grid in
// print_array's format (kernel.cu:115-129): '\n', then per row one char per cell ('0' if the cell
// equals 1, ' ' otherwise) and '\n', then a final '\n'.
#pragma once

namespace mdfx {
int run_cli(int argc, char** argv, const char* default_stencil, const char* prog);
}
