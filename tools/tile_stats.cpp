// Host-only tile statistics of a Kuhn block (tile count, tile nodes T, T/N) for the FAST tiling.
// build: hipcc -O2 -std=c++17 -Iinclude tools/tile_stats.cpp civiwave-fem_amd/csrc/tiles.cpp -o /tmp/tile_stats
// usage: /tmp/tile_stats NX NY NZ MAX_NODES MAX_ELEMS   (CWF_TILE_ORDER=morton for the round-1 tiling)
#include <algorithm>
#include "../civiwave-fem_amd/csrc/cwf_internal.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>
namespace cwf { int build_tiles(const cwf_system_desc *d, HostTiles &out, uint32_t max_nodes, uint32_t max_elems, int corners); }
// usage (fan groups): /tmp/tile_stats NX NY NZ MAX_NODES GROUPS_PER_TILE g  (needs groups.cpp on the build line)
int main(int argc, char **argv)
{
    int nx = atoi(argv[1]), ny = atoi(argv[2]), nz = atoi(argv[3]);
    uint32_t mn = atoi(argv[4]), me = atoi(argv[5]);
    const int KUHN[6][4] = {{0,1,3,7},{0,1,5,7},{0,2,3,7},{0,2,6,7},{0,4,5,7},{0,4,6,7}};
    uint64_t A = nx + 1, B = ny + 1, C = nz + 1, N = A * B * C, E = 6ull * nx * ny * nz;
    std::vector<double> xyz(3 * N);
    for (uint64_t k = 0; k < C; ++k) for (uint64_t j = 0; j < B; ++j) for (uint64_t i = 0; i < A; ++i) {
        uint64_t n = (k * B + j) * A + i; xyz[3*n] = 0.1*i; xyz[3*n+1] = 0.1*j; xyz[3*n+2] = 0.1*k; }
    std::vector<uint32_t> conn(8 * E, 0xFFFFFFFFu);
    uint64_t e = 0;
    for (int k = 0; k < nz; ++k) for (int j = 0; j < ny; ++j) for (int i = 0; i < nx; ++i) {
        uint32_t cn[8]; for (int b = 0; b < 8; ++b) cn[b] = ((k + ((b >> 2) & 1)) * B + (j + ((b >> 1) & 1))) * A + (i + (b & 1));
        for (int t = 0; t < 6; ++t, ++e) for (int a = 0; a < 4; ++a) conn[8 * e + a] = cn[KUHN[t][a]]; }
    std::vector<float> gr(24 * E, 0.f), vol(E, 1.f);
    cwf_system_desc d{};
    d.element_gradients = gr.data(); d.element_volume = vol.data();
    d.node_count = N; d.element_count = E; d.element_connectivity = conn.data(); d.node_coords = xyz.data(); d.material_count = 1;
    if (argc > 6 && argv[6][0] == 'g')
    {
        cwf::GroupTiles gt;
        int st = cwf::build_group_tiles(&d, gt, me, mn, 1u << 20);
        double T = gt.tile_nodes.size();
        printf("groups: status %d N=%lu G=%u tiles=%u T=%.0f T/N=%.3f nn_avg=%.1f max_nn=%u max_slots=%u\n", st, N,
               gt.ngroups, gt.ntiles, T, T / N, T / gt.ntiles, gt.max_tile_nodes, gt.max_tile_slots);
        // extra LDS cycles (bank conflicts) of the group phase's slot reads and pushes, per the lane-group
        // rules of MI355X_MICROARCH.md §LDS, summed over tiles (one wave-instruction per slot and wave)
        const int nt = (int)me;
        double rd128 = 0, rd64 = 0, rd16 = 0, wr64 = 0, wr32 = 0;
        auto lg128 = [](int l) { int h = (l & 63) >= 32 ? 2 : 0; l &= 31; bool g0 = l < 4 || (l >= 12 && l < 16) || (l >= 20 && l < 28); return h + (g0 ? 0 : 1); };
        for (uint32_t t = 0; t < gt.ntiles; ++t)
        {
            const uint32_t g0 = gt.hdr[t].x, ng = gt.hdr[t].y, nb = gt.hdr[t].z;
            for (int s = 0; s < 8; ++s)
            {
                // per lane group: distinct addresses per bank
                std::vector<std::vector<uint32_t>> a128(64 * 16), a64(64 * 64), a16(64 * 32), w64(64 * 32), w32(64 * 32);
                for (uint32_t L = 0; L < ng; ++L)
                {
                    const auto &g = gt.grec[g0 + L];
                    const uint32_t w = s < 3 ? g.x : s < 6 ? g.y : g.z, lid = (w >> (9 * (s % 3))) & 0x1ffu;
                    const uint32_t run = gt.run[nb + lid] & 0xffffu, q = run + ((g.w >> (4 * s)) & 15u);
                    const int wave = L / 64, G128 = wave * 4 + lg128(L), G32 = wave * 2 + (L & 63) / 32, G16 = wave * 4 + (L & 63) / 16;
                    auto add = [](std::vector<uint32_t> &v, uint32_t x) { if (std::find(v.begin(), v.end(), x) == v.end()) v.push_back(x); };
                    add(a128[G128 * 16 + (lid & 15)], lid);
                    add(a64[G32 * 64 + (2 * lid) % 64], lid);          // b64: bank (8 lid / 4) mod 64, 2 banks
                    add(a16[G32 * 32 + (lid / 2) % 32], lid / 2);      // u16: dword lid / 2, bank mod 32
                    add(w64[G16 * 32 + (2 * q) % 32], q);              // ds_write_b64 4 x 16: bank (8 q / 4) mod 32
                    add(w32[G32 * 32 + q % 32], q);                    // ds_write_b32 2 x 32
                }
                auto extra = [](std::vector<std::vector<uint32_t>> &v, int per) {
                    double e = 0; for (size_t i = 0; i < v.size(); i += per) { size_t m = 0; for (int k = 0; k < per; ++k) m = std::max(m, v[i + k].size()); if (m) e += m - 1; } return e; };
                rd128 += extra(a128, 16); rd64 += extra(a64, 64); rd16 += extra(a16, 32); wr64 += extra(w64, 32); wr32 += extra(w32, 32);
            }
        }
        printf("extra LDS cycles (group phase, whole mesh): read b128 %.0f  read b64 %.0f  read u16 %.0f  push b64 %.0f  push b32 %.0f\n",
               rd128, rd64, rd16, wr64, wr32);
        return 0;
    }
    cwf::HostTiles ht;
    cwf::build_tiles(&d, ht, mn, me, 4);
    double T = ht.tile_nodes.size();
    printf("N=%lu E=%lu tiles=%u T=%.0f T/N=%.3f nn_avg=%.1f ne_avg=%.1f max_nn=%u\n", N, E, ht.ntiles, T, T / N, T / ht.ntiles, (double)E / ht.ntiles, ht.max_tile_nodes);
}
