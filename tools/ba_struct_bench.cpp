// CPU timing of the local BA host structure (csrc/ba_structure.h) on a problem file written by
//   python3 tools/ba_struct_bench.py (C5 by default).  Build:
//   g++ -O2 -std=c++17 -Iinclude -Iorb-slam3_byzyh_amd/csrc tools/ba_struct_bench.cpp -o build/ba_struct_bench
#include <chrono>
#include <cstdio>
#include <vector>

#include "ba_structure.h"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int32_t hdr[3];
    if (fread(hdr, 4, 3, f) != 3) return 2;
    const int np = hdr[0], nq = hdr[1], ne = hdr[2];
    std::vector<double> pose(7 * (size_t)np), point(3 * (size_t)nq);
    std::vector<int64_t> pid(np), qid(nq);
    std::vector<uint8_t> fixed(np);
    std::vector<orb_ba_edge_t> edges(ne);
    bool ok = fread(pose.data(), 8, pose.size(), f) == pose.size() && fread(pid.data(), 8, np, f) == (size_t)np &&
              fread(fixed.data(), 1, np, f) == (size_t)np && fread(point.data(), 8, point.size(), f) == point.size() &&
              fread(qid.data(), 8, nq, f) == (size_t)nq && fread(edges.data(), sizeof(orb_ba_edge_t), ne, f) == (size_t)ne;
    fclose(f);
    if (!ok) return 2;
    orb_ba_problem_t pr{np, nq, ne, pose.data(), pid.data(), fixed.data(), nullptr, point.data(), qid.data(), edges.data()};
    orbgpu_ba::BaStructure S;
    using clk = std::chrono::steady_clock;
    double best = 1e9;
    for (int rep = 0; rep < 200; ++rep) {
        const auto t0 = clk::now();
        orbgpu_ba::ba_build_structure(&pr, 1, 0, S);
        const double us = std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        if (us < best) best = us;
    }
    printf("structure: %.1f us (best of 200); nf %d nl %d ne %d free edges %d blocks %d products <= %lld\n", best, S.nf,
           S.nl, S.ne, S.nfe, S.nblk, S.n_products);
    return 0;
}
