import sys, os, numpy as np, torch
sys.path[:0] = ['tests', 'safelife-k2_amd']
from test_gpu_board_planes import _pair, _host_planes
dev = torch.device('cuda:0')
B = 512
a, b = _pair((torch, dev), B, seed=99, tl=12)
rng = np.random.RandomState(5)
for t in range(3):
    acts = torch.from_numpy(rng.randint(0, 9, size=B).astype(np.int32)).to(dev)
    a.step_async(acts); b.step_async(acts)
    same = torch.equal(a.reward, b.reward)
    pok = a.planes_ok.cpu().numpy()
    bp = a.board_planes.cpu().numpy().view(np.uint32)
    bb = b.board.cpu().numpy()
    raw = a._board.cpu().numpy()
    ax = a.st_t['agent_x'].cpu().numpy(); ay = a.st_t['agent_y'].cpu().numpy()
    bad = []
    for e in range(B):
        if not (pok[e] & 64):
            continue
        hp = _host_planes(bb[e]); dp = bp[e].copy()
        for y, x in zip(*np.nonzero(bb[e] & 0x100)):
            k = 9 + 16 * (x & 1)
            hp[y >> 5, k, x >> 1] &= ~np.uint32(1 << (y & 31)); dp[y >> 5, k, x >> 1] &= ~np.uint32(1 << (y & 31))
        if not np.array_equal(hp, dp):
            d = np.nonzero(hp != dp)
            cells = set()
            for tt, k, j in zip(*d):
                diff = int(hp[tt, k, j] ^ dp[tt, k, j])
                for r in range(32):
                    if diff >> r & 1:
                        cells.add((32 * tt + r, 2 * j + (k >> 4), k & 15))
            bad.append((e, int(ax[e]), int(ay[e]), sorted(cells)[:6]))
    # u16 rows that must be valid: edges and the plus cells
    ubad = []
    for e in range(B):
        if not (pok[e] & 64) or (pok[e] & 128):
            continue
        for y in (0, 31, 32, 63, 64, 95, 96, 127):
            if not np.array_equal(raw[e, y], bb[e, y]):
                m = np.nonzero(raw[e, y] != bb[e, y])[0]
                if any(not (bb[e, y, x] & 0x100) for x in m):
                    ubad.append((e, 'edge', y, list(m[:4])))
        if not np.array_equal(raw[e, ay[e]], bb[e, ay[e]]):
            ubad.append((e, 'agent row', int(ay[e])))
        for d in (-2, -1, 1, 2):
            y = (ay[e] + d) % 128
            if raw[e, y, ax[e]] != bb[e, y, ax[e]]:
                ubad.append((e, 'col', int(y), int(ax[e])))
    print('t', t, 'rewards same', same, 'plane mismatches', len(bad), bad[:4], 'u16 mismatches', len(ubad), ubad[:6])
