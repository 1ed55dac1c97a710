#!/usr/bin/env python3
"""Tet evaluations per tet of the PARITY node tiles: strips of 256 consecutive nodes against the compact
breadth-first tiles abi.cpp:parity_compact_tiles builds (the same greedy algorithm, restated on the host).
usage: tools/parity_tile_factor.py [config]   (C2: strip 2.277, compact 1.489)"""
import sys, numpy as np
sys.path.insert(0,'civiwave-fem_amd')
from cwf import scenarios
case = scenarios.config_case(sys.argv[1] if len(sys.argv) > 1 else 'c2')
P = case.packing
conn = np.asarray(P.connectivity, dtype=np.int64).reshape(-1,8)[:, :4]
N = P.node_count; E = conn.shape[0]
off = np.asarray(P.offsets, dtype=np.int64); inc = np.asarray(P.element_indices, dtype=np.int64)
# strip factor
def factor(tiles):
    tot = 0
    for t in tiles:
        ts = set()
        for n in t:
            ts.update(inc[off[n]:off[n+1]].tolist())
        tot += len(ts)
    return tot / E
strips = [range(b, min(N, b+256)) for b in range(0, N, 256)]
# BFS compact
state = np.zeros(N, np.int8); tiles = []
offl = off.tolist(); incl = inc.tolist(); connl = conn.tolist()
for seed in range(N):
    if state[seed]: continue
    q = [seed]; state[seed] = 1; head = 0; placed = []
    while head < len(q) and len(placed) < 256:
        u = q[head]; head += 1; state[u] = 2; placed.append(u)
        for j in range(offl[u], offl[u+1]):
            for v in connl[incl[j]]:
                if not state[v]:
                    state[v] = 1; q.append(v)
    for v in q[head:]: state[v] = 0
    tiles.append(placed)
sizes = np.array([len(t) for t in tiles])
print("N", N, "E", E, "strips", len(strips), "compact", len(tiles), "mean size %.1f" % sizes.mean(), "tiles<128:", (sizes < 128).sum())
print("factor strip %.3f compact %.3f" % (factor(strips), factor(tiles)))
