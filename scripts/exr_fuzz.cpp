// Sanitizer harness for host/exr_read.cpp: decode every file named on the command line
// (build: g++ -g -O1 -fsanitize=address,undefined scripts/exr_fuzz.cpp raytracer-795_amd/host/exr_read.cpp -lz).
#include <cstdio>
#include <string>
#include <vector>

#include "../raytracer-795_amd/host/exr_read.hpp"

int main(int argc, char** argv) {
    int ok = 0, bad = 0;
    for (int i = 1; i < argc; i++) {
        std::vector<float> rgba;
        int w = 0, h = 0;
        std::string err;
        if (rtgh::read_exr_rgba(argv[i], rgba, w, h, err)) ok++; else bad++;
    }
    printf("decoded %d, rejected %d\n", ok, bad);
    return 0;
}
