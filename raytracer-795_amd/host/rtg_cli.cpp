// rtg_cli — the reference's command line (`./raytracer scene.xml`, src/main.cpp:7-14) on the
// MI355X path: parse the scene (rtgh_parse_xml), build it on the GPU, render and save every
// camera (rtgh_render_scene).
//
//   rtg_cli scene.xml [--device N] [--devices G] [--seed S] [--out-dir DIR]
//
// --devices G renders every camera on G GPUs (device N and the next G-1): one host thread per
// GPU, row-block pixel shards, RCCL gather of the rows onto device N -- the reference's
// renderScene fork over 8 std::threads (src/Scene.cpp:294-363, threads at 340-356) moved to GPUs.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/rtg_host.h"

int main(int argc, char** argv) {
    const char* xml = nullptr;
    const char* out_dir = nullptr;
    int device = 0, devices = 0;
    unsigned long long seed = 0x5EED2026ull;
    for (int i = 1; i < argc; i++) {
        if (!strcmp(argv[i], "--device") && i + 1 < argc) device = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--devices") && i + 1 < argc) devices = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--seed") && i + 1 < argc) seed = strtoull(argv[++i], nullptr, 0);
        else if (!strcmp(argv[i], "--out-dir") && i + 1 < argc) out_dir = argv[++i];
        else if (argv[i][0] == '-') { fprintf(stderr, "unknown option %s\n", argv[i]); return 2; }
        else xml = argv[i];
    }
    if (!xml) {
        fprintf(stderr, "usage: %s scene.xml [--device N] [--devices G] [--seed S] [--out-dir DIR]\n", argv[0]);
        return 2;
    }
    const int rc = rtgh_render_scene_multi(xml, device, devices, seed, out_dir);
    if (rc != RTG_OK) {
        fprintf(stderr, "rtg_cli: %s\n", rtgh_last_error());
        return 1;
    }
    return 0;
}
