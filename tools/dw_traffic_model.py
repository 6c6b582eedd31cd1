"""L2-miss (fabric) traffic model of the 8-wave GEMM's tile schedule, to read the PMC FETCH_SIZE
records against (profiles/roofline_traffic.json). Each XCD has its own 4 MB L2 and runs 32 tiles
at a time (one 512-thread block per CU); its concurrent tiles stream their A and B panels
(256 rows x K) through the K loop roughly in lockstep, so an XCD fetches every DISTINCT panel of
its concurrent tiles once per round and nothing carries over between rounds (a round's panels
are K x 0.5 KB each, far beyond 4 MB). Blocks go to XCDs round-robin (b % 8) in dispatch order;
tile order = gemm.hip's xcd_remap + tile_origin (groups of 4 N-tiles sweeping M by default).

  python tools/dw_traffic_model.py
"""


def cdiv(a, b):
    return -(-a // b)


def xcd_remap(bid, nwg):
    q, r, x = nwg // 8, nwg % 8, bid % 8
    return (x * (q + 1) if x < r else r * (q + 1) + (x - r) * q) + bid // 8


def tile_origin(lid, tiles_m, tiles_n, group):
    if group < 0:
        gn = -group
        per = gn * tiles_m
        g = lid // per
        first = g * gn
        gs = min(tiles_n - first, gn)
        return (lid % per) // gs, first + (lid % per) % gs
    per = group * tiles_n
    g = lid // per
    first = g * group
    gs = min(tiles_m - first, group)
    return first + (lid % per) % gs, (lid % per) // gs


def traffic(M, N, K, bm=256, bn=256, cus=256, group=-4):
    tm, tn = cdiv(M, bm), cdiv(N, bn)
    nwg = tm * tn
    total = 0
    for r0 in range(0, nwg, cus):
        per_xcd = {}
        for b in range(r0, min(nwg, r0 + cus)):
            m, n = tile_origin(xcd_remap(b, nwg), tm, tn, group)
            a_set, b_set = per_xcd.setdefault(b % 8, (set(), set()))
            a_set.add(m)
            b_set.add(n)
        for a_set, b_set in per_xcd.values():
            total += (len(a_set) * bm + len(b_set) * bn) * K * 2
    return total + M * N * 2  # + C written once


def main():
    # the config-3 dW launches of one step (M x N x K of dW = dY^T X) and the bench's 22 extra
    # lm_head-shape launches in the profiled pass (library ceiling), as in the PMC record
    T = 8704
    mix = [((12288, 4096, T), 32), ((4096, 4096, T), 32), ((22016, 4096, T), 32), ((4096, 11008, T), 32),
           ((32064, 4096, T), 1), ((4096, 4096, 4608), 1)]
    tot_model = tot_alg = n = 0
    for (M, N, K), cnt in mix:
        t = traffic(M, N, K)
        alg = (M * K + N * K + M * N) * 2
        print(f"dW {M}x{N}x{K}: model {t / 1e9:.3f} GB/launch, algorithmic {alg / 1e9:.3f} GB ({t / alg:.2f}x)")
        tot_model += t * cnt
        tot_alg += alg * cnt
        n += cnt
    print(f"step mix (2 profiled steps + 22 ceiling launches weighted as in the record): ", end="")
    extra = traffic(32064, 4096, T) * 22
    print(f"model {(2 * tot_model + extra) / (2 * n + 22) / 1e9:.3f} GB/launch, algorithmic "
          f"{(2 * tot_alg + 22 * (32064 * T + 4096 * T + 32064 * 4096) * 2) / (2 * n + 22) / 1e9:.3f} GB/launch")


if __name__ == "__main__":
    main()
