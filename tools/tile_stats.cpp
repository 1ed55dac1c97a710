// Host-only tile statistics of a Kuhn block (tile count, tile nodes T, T/N) for the FAST tiling.
// build: hipcc -O2 -std=c++17 -Iinclude tools/tile_stats.cpp civiwave-fem_amd/csrc/tiles.cpp -o /tmp/tile_stats
// usage: /tmp/tile_stats NX NY NZ MAX_NODES MAX_ELEMS   (CWF_TILE_ORDER=morton for the round-1 tiling)
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
        return 0;
    }
    cwf::HostTiles ht;
    cwf::build_tiles(&d, ht, mn, me, 4);
    double T = ht.tile_nodes.size();
    printf("N=%lu E=%lu tiles=%u T=%.0f T/N=%.3f nn_avg=%.1f ne_avg=%.1f max_nn=%u\n", N, E, ht.ntiles, T, T / N, T / ht.ntiles, (double)E / ht.ntiles, ht.max_tile_nodes);
}
