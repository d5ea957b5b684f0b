"""Where the VALU instructions of the two profiled passes go, from their plans and their ISA.

    python tools/overhead_accounting.py deep   [--resident 3072] [--sq-valu 300.27e6]   # 65536^2 torus (12, 2) pass
    python tools/overhead_accounting.py coop   [--sq-valu 158.2e6 --sq-salu 89.25e6]     # config 2: 4096^2 cooperative

Prints one JSON object: the modelled SQ_INSTS_VALU per launch, split into what B3/S23 needs and each overhead the
plan adds, next to the measured counter (profiles/r5/final/pmc_sq_*.json, device code c2ddb3d36af2fd90).

deep: mirrors plan_stream (csrc/gol_step.hip) for one balanced round of `resident` waves (256 CUs x 12 waves at the
(12, 2) pass's 3 waves per SIMD): 16 seam strips of 63 blocks + 16 remainder blocks per 65536-cell row, 62 group
segments of 1058 rows (the last 998), three waves per SIMD group splitting a segment by the split / split2 shares
(group_cut), the remainder blocks packed 3 sub-strips per wave.  Per wave: ceil((share + 2K) / 4) trips of 4 rows;
the first 6 trips are pipeline fill, where level g runs only if the trip holds a row at step >= 2g.  VALU per trip
from the ISA of gol_stream_step<12, 2, false, true, 0> (hipcc -O3 -S, round-6 build):
    steady loop (2 trips, 96 level-rows):  2130 VALU = 1728 v_bitop3 (18 per level-row) + 192 DPP + 192 v_alignbit
                                           + 16 seam merges (v_bitop3, one per word and row) + 2 other
    fill loop (2 trips, up to 96 level-rows): 2341 VALU (the same + 178 v_mov / 25 v_cmp of the skip branches)
coop: the cooperative pass's block schedule (csrc/gol_coop.hip gol_band_pass<2, 2, 1, false, true>): 256 bands of
16 rows, K = 8, 16 waves x 2 rows, 1000 generations.  Per generation a wave runs the row sums (16 VALU) while a
producing neighbour reads them (j <= j_act), the rule (28 VALU) while it produces (j < j_act), and one LDS-address
VALU; per block it publishes and polls (the rest).
"""
from __future__ import annotations

import argparse
import json


def group_cut(length: int, i: int, n: int, k: int, split: float, split2: float) -> int:
    """csrc/gol_step.hip StreamWave::group_cut (float math as on the device)."""
    if i <= 0:
        return 0
    if i >= n:
        return length
    rho = (1.0 - split) / split
    rho2 = (1.0 - split2) / split2
    pw, s, head = 1.0, 0.0, 0.0
    for j in range(n):
        if j == i:
            head = s
        s += pw
        pw *= rho if j == 0 else rho2
    total = float(length + 2 * k * n)
    cut = int(total * head / s + 0.5) - 2 * k * i
    return max(0, min(length, cut))


def level_rows(share: int, k: int, r: int = 4):
    """(steady level-rows, fill level-rows, fill trips) of one wave streaming `share` rows at depth k."""
    nsteps = share + 2 * k
    ntrips = -(-nsteps // r)
    t_fill = min((2 * k) // r, ntrips)
    fill_trips = (t_fill // 2) * 2
    fill = steady = 0
    for t in range(ntrips):
        for g in range(k):
            skip = t < fill_trips and t * r + r - 1 < 2 * g
            if skip:
                continue
            if t < fill_trips:
                fill += r
            else:
                steady += r
    return steady, fill, fill_trips


def deep(args) -> dict:
    W = H = 65536
    k, m = 12, 2
    words = W // 32
    nblocks = words // m
    kseam = 63
    nstrips = nblocks // kseam
    rem = nblocks - nstrips * kseam
    rem_p = 64 // (rem + 2)
    group = 3
    slots = args.resident // group
    per_seg = nstrips + (1.0 / rem_p if rem else 0.0)
    nsegs = max(1, int(slots / per_seg))
    seg = -(-H // nsegs)
    nsegs = -(-H // seg)
    over = (-(-(seg + 2 * k) // 4) + 1) * 4 - (seg + 2 * k)
    rem_mid = max(0, min(nsegs - 2, (H - k - over) // seg - 1))
    packed = -(-rem_mid // rem_p)
    rem_units = 1 + packed + (nsegs - 1 - rem_mid)
    steady_per_lr = 2130 / 96.0
    fill_per_lr = 2341 / 96.0
    # every unit (a strip's segment or a remainder unit) is one SIMD group of three waves over one segment
    seg_len = [seg] * (nsegs - 1) + [H - seg * (nsegs - 1)]
    units = [(s, "main") for s in seg_len for _ in range(nstrips)]
    units += [(seg_len[0], "rem")] + [(seg, "rem")] * packed + [(s, "rem") for s in seg_len[1 + rem_mid:]]
    valu = 0.0
    lr_total = 0
    for s, _ in units:
        for role in range(group):
            share = group_cut(s, role + 1, group, k, args.split, args.split2) - group_cut(s, role, group, k, args.split,
                                                                                          args.split2)
            st, fi, _ = level_rows(share, k)
            valu += st * steady_per_lr + fi * fill_per_lr
            lr_total += st + fi
    wave_word_gens = W * H / 32 / 64 * k
    useful_lr = nblocks * H * k / 64  # level-rows if every lane held a useful block and no row were recomputed
    ideal = 11.0 * wave_word_gens
    out = {
        "pass": "gol_stream_step<12, 2, false, true> on 65536^2 torus (the headline launch)",
        "plan": {"resident_waves": args.resident, "waves_used": len(units) * group, "seam_strips": nstrips,
                 "remainder_blocks": rem, "subs_per_remainder_wave": rem_p, "segments": nsegs, "segment_rows": seg,
                 "remainder_units": rem_units, "split": args.split, "split2": args.split2},
        "valu_per_wave_word_gen": {
            "designed (9 v_bitop3 + per block of 2 words 2 DPP + 2 v_alignbit)": 11.0,
            "steady loop (adds the seam merge)": round(steady_per_lr / 2, 3),
            "modelled launch": round(valu / wave_word_gens, 3),
            "measured (SQ_INSTS_VALU)": round(args.sq_valu / wave_word_gens, 3) if args.sq_valu else None,
        },
        "level_rows": {"executed": lr_total, "useful_equivalent": useful_lr},
        "ideal_sq_valu": ideal,
        "modelled_sq_valu": valu,
    }
    # split the modelled excess over the ideal into its causes
    lanes_useful = nblocks / ((nstrips + rem_units / nsegs) * 64)  # useful blocks per lane launched, per row
    halo_rows = 0
    for s, _ in units:
        for role in range(group):
            share = group_cut(s, role + 1, group, k, args.split, args.split2) - group_cut(s, role, group, k, args.split,
                                                                                          args.split2)
            st, fi, _ = level_rows(share, k)
            halo_rows += st + fi - share * k
    rows_lr = lr_total - halo_rows
    fill_lr = sum(level_rows(group_cut(s, r + 1, group, k, args.split, args.split2) -
                             group_cut(s, r, group, k, args.split, args.split2), k)[1]
                  for s, _ in units for r in range(group))
    out["overheads_pct_of_designed"] = {
        "seam merge (1 v_bitop3 per word and row, at level 0)": round(100 * (steady_per_lr / 22 - 1), 2),
        "recomputed halo rows (about K (K + 1) level-rows per wave)": round(100 * halo_rows / rows_lr, 2),
        "lanes without a useful block (seam lane, remainder waves' idle lanes, halo lanes)":
            round(100 * (1 / lanes_useful - 1), 2),
        "fill-loop v_mov / v_cmp (skip branches)": round(100 * fill_lr * (fill_per_lr - steady_per_lr) / valu, 2),
    }
    return out


def coop(args) -> dict:
    K, B, R, NW, gens = 8, 16, 2, 16, 1000
    tot = {"row sums (16 VALU while a producing neighbour reads them)": 0,
           "rule (28 VALU while the wave produces rows)": 0, "LDS slot address (1 VALU)": 0}
    for blk in range(-(-gens // K)):
        k = min(K, gens - blk * K)
        for j in range(k):
            for wv in range(NW):
                r0 = wv * R
                j_act = min(K + B + k - 1 - r0, r0 + R - K + k - 1)
                tot["LDS slot address (1 VALU)"] += 1
                if j <= j_act:
                    tot["row sums (16 VALU while a producing neighbour reads them)"] += 16
                if j < j_act:
                    tot["rule (28 VALU while the wave produces rows)"] += 28
    wave_gens = 4096 * gens  # 256 bands x 16 waves
    per = {key: round(v * 256 / wave_gens, 2) for key, v in tot.items()}
    loop = sum(per.values())
    # rows computed per generation against the band's 16: the temporal block's shrinking halo
    computed = sum(max(0, (K + B + min(K, gens - b * K) - 1 - j) - (K - min(K, gens - b * K) + 1 + j))
                   for b in range(-(-gens // K)) for j in range(min(K, gens - b * K)))
    out = {
        "pass": "gol_band_pass<2, 2, 1, false, true>: 4096^2 torus, 1000 generations (BASELINE config 2)",
        "schedule": {"bands": 256, "band_rows": B, "K": K, "waves": NW, "rows_per_wave": R},
        "valu_per_wave_gen": dict(per, **{
            "generation loop, modelled": round(loop, 2),
            "measured (SQ_INSTS_VALU / 4096 waves / 1000 generations)": round(args.sq_valu / wave_gens, 2)
            if args.sq_valu else None}),
        "rows_computed_per_band_row": round(computed / (gens * B), 3),
        "b3s23_floor_valu_per_wave_gen": round(2 * 22 * B / NW / 2, 2),
    }
    if args.sq_valu:
        out["valu_per_wave_gen"]["outside the loop (publish, poll, load, store)"] = round(
            args.sq_valu / wave_gens - loop, 2)
    if args.sq_salu:
        out["salu_per_wave_gen"] = {
            "measured (SQ_INSTS_SALU)": round(args.sq_salu / wave_gens, 2),
            "generation loop (ISA: slot parity and address 5, loop and activity tests 5)": 10,
            "per block of 8 (ISA: granule addresses and tags, 64-bit products), per generation": 6,
        }
        out["salu_per_wave_gen"]["rest: poll rounds (s_sleep, tag test, loop)"] = round(
            args.sq_salu / wave_gens - 16, 2)
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("which", choices=["deep", "coop"])
    p.add_argument("--resident", type=int, default=3072)
    p.add_argument("--split", type=float, default=0.66)
    p.add_argument("--split2", type=float, default=0.76)
    p.add_argument("--sq-valu", type=float, default=None)
    p.add_argument("--sq-salu", type=float, default=None)
    a = p.parse_args()
    if a.which == "deep" and a.sq_valu is None:
        a.sq_valu = 300.27e6  # profiles/r5/final/pmc_sq_torus_k12.json, per launch
    if a.which == "coop" and a.sq_valu is None:
        a.sq_valu, a.sq_salu = 158196912.0, 89250784.0  # profiles/r5/final/pmc_sq_c2.json
    print(json.dumps(deep(a) if a.which == "deep" else coop(a), indent=1))


if __name__ == "__main__":
    main()
