"""DESIGN.md §4c, first-divergence localisation of the row-chain hazard.

Runs the config-2 sampler (J = 16, 3,200 rows) at T = 2 on the tiled split route twice -- one
row chain, then `chains` row chains -- with the diagnostic snapshot arena set
(sd_debug_snapshot): every graph-linear call copies its phase-1 scratch Y (k_gl4t output) and its
output (phase-2 output) into slot (step, call), the posterior update its output into the step's
last slot.  Prints the first slots where the two runs differ, where in the tile / node / column
grid the differences sit, and whether the differing values are another position's or an older
write's (addressing, lost stores) or new values (arithmetic).
Load the CU-sharing diagnostic build (SKELDIFF_LIB=.../libskeldiff_share.so) to reproduce.
HAZARD_DUMP=1 also dumps the inputs the first posterior update computed from (x0, x_t, sigma
eps: sd_debug_update_dump) and compares them between the two runs.
usage: python tools/hazard_snap.py [chains] [T]"""
import ctypes
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402
from skeletondiffusion_amd import _lib  # noqa: E402

chains = int(sys.argv[1]) if len(sys.argv) > 1 else 3
T = int(sys.argv[2]) if len(sys.argv) > 2 else 2
CALLS = 40  # kSnapCalls (sd_plan.hip)
dev = torch.device("cuda", 0)
d, xc, rows = bench.build_config("amass16", dev, T=T, batch=64)
eng = d.engine
J = d.channels
lib = _lib.lib()
lib.sd_debug_snapshot.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]
lib.sd_debug_snapshot_meta.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
lib.sd_debug_update_dump.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
DUMP = os.environ.get("HAZARD_DUMP") == "1"  # the first update's inputs (sd_debug_update_dump)
dumps = {}
YF = rows * J * 768
SLOT = YF + rows * J * 256
NS = T * CALLS


def run(nch):
    eng.set_option("split_route", 3)
    eng.set_option("row_chains", nch)
    arena = torch.zeros(NS * SLOT, device=dev)
    out = torch.empty((rows, J, 96), device=dev)
    eng.sample_loop(rows, x_cond=xc, seed=77, row0=0, graph=False, out=out, keep_start=False)  # plan + warm
    torch.cuda.synchronize()
    lib.sd_debug_snapshot(arena.data_ptr(), SLOT, YF, NS)
    if DUMP:
        dm = torch.full((3, rows, J, 96), float("nan"), device=dev)
        lib.sd_debug_update_dump(dm[0].data_ptr(), dm[1].data_ptr(), dm[2].data_ptr())
    eng.sample_loop(rows, x_cond=xc, seed=77, row0=0, graph=False, out=out, keep_start=False)
    torch.cuda.synchronize()
    if DUMP:
        lib.sd_debug_update_dump(None, None, None)
        dumps[nch] = dm
    meta = []
    for s in range(NS):
        m = (ctypes.c_int32 * 3)()
        lib.sd_debug_snapshot_meta(s, m)
        meta.append(tuple(m))
    lib.sd_debug_snapshot(None, 0, 0, 0)
    st = eng.status(rows)
    return arena, out.clone(), meta, st


A, outA, metaA, stA = run(1)
B, outB, metaB, stB = run(chains)
print(f"status words: 1 chain {stA:#x}, {chains} chains {stB:#x}")
print(f"final latents: max|d| = {(outA - outB).abs().max().item():.3e}, "
      f"differing rows {int((outA != outB).flatten(1).any(1).sum())} of {rows}")
bounds = [(rows // 32) * i // chains * 32 for i in range(chains)] + [rows]


def chain_of(r):
    for i in range(chains):
        if bounds[i] <= r < bounds[i + 1]:
            return i
    return -1


def describe_y(idx, N):
    """Y scratch layout [tile][node][32 rows][N] -> (row, node, col)"""
    col = idx % N
    r = (idx // N) % 32
    node = (idx // (32 * N)) % J
    tile = idx // (32 * N * J)
    return tile * 32 + r, node, col


def describe_blk(idx, F):
    """row-blocked layout [row block][node][F/8][2][32][4] -> (row, node, feature)"""
    rb = idx // (J * F * 32)
    node = (idx // (F * 32)) % J
    rem = idx % (F * 32)
    f = (rem // 256) * 8 + ((rem // 128) & 1) * 4 + rem % 4
    r = (rem // 4) % 32
    return rb * 32 + r, node, f


shown = 0
for s in range(NS):
    step, call = divmod(s, CALLS)
    N, out_rs, yrow = metaB[s]
    for region, lo, hi in (("Y", 0, YF), ("out", YF, SLOT)):
        a = A[s * SLOT + lo: s * SLOT + hi]
        b = B[s * SLOT + lo: s * SLOT + hi]
        ne = (a != b).nonzero().flatten()
        if ne.numel() == 0:
            continue
        dmax = (a - b).abs().max().item()
        print(f"\n== step {step} call {call} ({'update' if call == CALLS - 1 else f'N={N}'}) region {region}: "
              f"{ne.numel()} differing floats, max|d| = {dmax:.3e}")
        idx = ne[:200000].cpu()
        if region == "Y":
            rr, nn, cc = describe_y(idx, N)
            wg = set(zip((rr // 128).tolist(), nn.tolist(), (cc // 192).tolist()))
            waves = set(zip((rr // 32).tolist(), nn.tolist()))
            print(f"   k_gl4t work units hit: {len(wg)} (row group, node, col group); (tile, node) waves: {len(waves)}")
            print(f"   rows by chain: {[sum(1 for r in set(rr.tolist()) if chain_of(r) == i) for i in range(chains)]}, "
                  f"nodes {sorted(set(nn.tolist()))}, cols {cc.min().item()}..{cc.max().item()}")
            print(f"   first units: {sorted(wg)[:8]}")
        elif call == CALLS - 1:
            rr = idx // (J * 96)
            nn = (idx // 96) % J
            dd = idx % 96
            print(f"   update rows by chain: {[sum(1 for r in set(rr.tolist()) if chain_of(r) == i) for i in range(chains)]}")
            # per bad row: which nodes i differ, and in how many of the 96 features
            per = {}
            for r, n_, f_ in zip(rr.tolist(), nn.tolist(), dd.tolist()):
                per.setdefault(r, {}).setdefault(n_, set()).add(f_)
            shapes = {}
            for r, m in per.items():
                key = tuple(sorted((n_, len(fs)) for n_, fs in m.items()))
                shapes[key] = shapes.get(key, 0) + 1
            top = sorted(shapes.items(), key=lambda kv: -kv[1])[:8]
            print(f"   per-row pattern ((node, features differing), ...): count -> {top}")
            wgs = {}
            for r, m in per.items():  # k_update workgroup = 256 threads = 256 / 48 rows of the chain
                c = chain_of(r)
                wgs.setdefault((c, ((r - bounds[c]) * 48) // 256), set()).update(m.keys())
            print(f"   update workgroups hit: {len(wgs)}; nodes per workgroup: "
                  f"{sorted((k, sorted(v)) for k, v in wgs.items())[:10]}")
        else:
            F = out_rs // J
            if call == 34:  # final_glin: row-major x0
                rr = idx // (J * F)
                nn = (idx // F) % J
            else:
                rr, nn, _ = describe_blk(idx, F)
            print(f"   rows by chain: {[sum(1 for r in set(rr.tolist()) if chain_of(r) == i) for i in range(chains)]}, "
                  f"nodes {sorted(set(nn.tolist()))}, distinct rows {len(set(rr.tolist()))}")
        # provenance of the differing values (first 4096)
        k = ne[:4096]
        bad = b[k]
        same_slot = torch.isin(bad, a).float().mean().item()
        prev = B[(s - 1) * SLOT + lo: (s - 1) * SLOT + hi][k] if s > 0 else None
        older = (bad == prev).float().mean().item() if prev is not None else float("nan")
        rel = ((bad - a[k]).abs() / a[k].abs().clamp_min(1e-30)).median().item()
        print(f"   bad values: {same_slot:.3f} occur elsewhere in the 1-chain slot; {older:.3f} equal the previous "
              f"call's value at that address (lost write); median rel. error {rel:.2e}")
        print(f"   samples (1-chain, {chains}-chain): {[(round(x, 6), round(y, 6)) for x, y in zip(a[k[:4]].tolist(), bad[:4].tolist())]}")
        shown += 1
    if shown >= 6:
        break
if shown == 0:
    print("no differing slot")

if DUMP:
    a, b = dumps[1], dumps[chains]
    for q, name in enumerate(("x0 (act + clamp)", "x_t", "sigma eps")):
        ne = (a[q] != b[q]).nonzero()
        print(f"\n== first update's input {name}: {ne.shape[0]} differing floats (NaN = not written: "
              f"{int(torch.isnan(b[q]).sum())})")
        if ne.shape[0] == 0:
            continue
        rr, nn, ff = ne[:, 0], ne[:, 1], ne[:, 2]
        g = rr * 48 + ff // 2  # thread index of the chain-0-relative grid ~ (row, feature pair)
        lanes = set(((rr * 48 + ff // 2) % 64 // 8).tolist())
        print(f"   rows by chain {[sum(1 for r in set(rr.tolist()) if chain_of(r) == i) for i in range(chains)]}, "
              f"nodes {sorted(set(nn.tolist()))[:16]}, 8-lane groups {sorted(lanes)}")
        runs = {}
        for r, f_ in set(zip(rr.tolist(), (ff // 16).tolist())):
            runs[(r, f_)] = runs.get((r, f_), 0) + 1
        print(f"   (row, 16-feature block) units: {len(runs)}; first {sorted(runs)[:10]}")
        k = ne[:4096]
        bad = b[q][k[:, 0], k[:, 1], k[:, 2]]
        good = a[q][k[:, 0], k[:, 1], k[:, 2]]
        print(f"   samples (right, wrong): {[(round(x, 6), round(y, 6)) for x, y in zip(good[:6].tolist(), bad[:6].tolist())]}")
        print(f"   wrong values found in the same dump (1 chain): {torch.isin(bad, a[q]).float().mean().item():.3f}; "
              f"in the other inputs: {[round(torch.isin(bad, a[z]).float().mean().item(), 3) for z in range(3)]}")
        hits = []
        for arena, lab in ((A, "1-chain"), (B, f"{chains}-chain")):
            for sl in range(NS):
                for region, lo, hi in (("Y", 0, YF), ("out", YF, SLOT)):
                    fr = torch.isin(bad, arena[sl * SLOT + lo: sl * SLOT + hi]).float().mean().item()
                    if fr > 0.05:
                        hits.append((lab, sl // CALLS, sl % CALLS, region, round(fr, 3)))
        print(f"   wrong values found in the snapshot slots (run, step, call, region, fraction): {hits[:20]}")
