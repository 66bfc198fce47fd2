#!/usr/bin/env python3
"""Round 5: the xN decoders' frac-vs-N table from tools/r5_curve.sh (bench lines)
and tools/r5_curve_pmc.sh (PMC passes + kernel trace):
    python3 tools/r5_curve_table.py gpurun_out > profiles/r05_dec_curve.txt"""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
N_IN = 1 << 28


def pmc(path, counter):
    for f in glob.glob(os.path.join(path, "*_counter_collection.csv")):
        vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                if r["Counter_Name"] == counter and "k_dec_xn" in r["Kernel_Name"]]
        if vals:
            return sum(vals) / len(vals)
    return None


def trace_avg(path):
    for f in glob.glob(os.path.join(path, "*_kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if "k_dec_xn" in r["Name"]:
                return float(r["AverageNs"]) / 1e3
    return None


print("One 256 MiB uniform buffer, N streams. frac = (C + N_in) / decoder time / 8 TB/s;")
print("bench: timed-region event average; trace: rocprofv3 kernel-trace average over the")
print("profiled run (warm-up and instrumented passes included). Per wave-step = per")
print("symbol per wave (2^28 / 64 wave-steps). FETCH_SIZE x2 (gfx950 rule) over C.")
print()
hdr = ("N", "decoder", "bench us", "frac", "trace us", "VALU/ws", "SALU/ws", "LDS/ws", "bankconf/ws",
       "WAIT_ANY%", "WAIT_INST%", "FETCH/C", "WRITE MB")
print(" | ".join(hdr))
for N in (1 << 18, 1 << 19, 1 << 20):
    for R, name in ((1, "k_dec_xn_fast (VGPR ring, 4 waves/SIMD)"), (2, "k_dec_xn_dma (DMA ring, 8 waves/SIMD)")):
        bj = os.path.join(root, f"r5_curve_{N}_{R}.json")
        try:
            line = json.loads(open(bj).read().strip().splitlines()[-1])
            rd = line["roofline_decode"]
            C = line["compressed_bytes"]
            bus, frac = rd["avg_launch_ms"] * 1e3, rd["frac"]
        except Exception:
            continue
        p = os.path.join(root, "r5_pmc", f"n{N}_r{R}")
        ws = N_IN / 64
        v = pmc(p + "_sq1", "SQ_INSTS_VALU")
        sa = pmc(p + "_sq1", "SQ_INSTS_SALU")
        wc = pmc(p + "_sq1", "SQ_WAVE_CYCLES")
        wa = pmc(p + "_sq1", "SQ_WAIT_ANY")
        wi = pmc(p + "_sq1", "SQ_WAIT_INST_ANY")
        ld = pmc(p + "_sq2", "SQ_INSTS_LDS")
        bc = pmc(p + "_sq2", "SQ_LDS_BANK_CONFLICT")
        fe = pmc(p + "_f", "FETCH_SIZE")
        wr = pmc(p + "_w", "WRITE_SIZE")
        tr = trace_avg(p + "_kt")
        f = lambda x, d=1: "-" if x is None else f"{x:.{d}f}"
        print(" | ".join([f"2^{N.bit_length() - 1}", name, f(bus), f"{frac:.3f}", f(tr),
                          f(v / ws if v else None), f(sa / ws if sa else None), f(ld / ws if ld else None),
                          f(bc / ws if bc else None), f(100 * wa / wc if wa else None, 0),
                          f(100 * wi / wc if wi else None, 0), f(fe * 1024 * 2 / C if fe else None, 2),
                          f(wr * 1024 / 1e6 if wr else None, 0)]))
