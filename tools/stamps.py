"""Per-workgroup phase breakdown of one x3 GEMM launch, from a diagnostic build with in-kernel stamps
(csrc/stamp.h; build it with tools/abvar.sh stamp -DX3_STAMP=1, run with CAPMI_LIB=ab/stamp.so).

python tools/stamps.py --shape l3c3 --x3d --dense   (every tools/gemm_one.py option)

Prints, over the launch's workgroups: the clock they ran at, the main loop's cycles per k-tile (first
segment of a workgroup apart: it includes the operand prologue), the epilogue, stream-K publish and
consume cycles, and the launch span against the sum of each workgroup's phases (the idle tail)."""
import ctypes
import os
import statistics as st
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402

from gemm_one import parser, setup  # noqa: E402
from capmi import _lib  # noqa: E402

SLOTS, BLOCKS = 64, 4096
EV = {1: "start", 2: "rstart", 3: "seg", 4: "main", 5: "pub", 6: "cons", 7: "epi", 8: "end", 9: "rend"}


def read(name):
    lib = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_ulonglong * (SLOTS * BLOCKS))()
    rc = getattr(lib, name + "_read")(buf, ctypes.c_longlong(SLOTS * BLOCKS))
    if rc:
        raise RuntimeError(f"{name}_read: {rc}")
    return buf


def clear(name):
    lib = ctypes.CDLL(_lib.LIB_PATH)
    rc = getattr(lib, name + "_clear")()
    if rc:
        raise RuntimeError(f"{name}_clear: {rc}")


def parse(buf):
    wgs = []
    for b in range(BLOCKS):
        recs = []
        for s in range(SLOTS):
            v = buf[b * SLOTS + s]
            if v == 0:
                break
            code = v >> 48
            recs.append((code & 0xff, code >> 8, v & 0xffffffffffff))
        if recs:
            wgs.append(recs)
    return wgs


def analyse(wgs):
    per_kt, first_kt, epi, pub, cons, span, mhz, busy, tstart, tend, segs = [], [], [], [], [], [], [], [], [], [], []
    for recs in wgs:
        d = {}
        cur = None
        first = True
        t_prev = None
        for ev, arg, t in recs:
            name = EV.get(ev, "?")
            if name in ("start", "end", "rstart", "rend"):
                d[name] = t
                if name == "start":
                    t_prev = t
                continue
            if name == "seg":
                cur = (t, arg)
                segs.append(arg)
            elif name == "main" and cur is not None:
                (first_kt if first else per_kt).append((t - cur[0]) / max(cur[1], 1))
                first = False
                t_prev = t
            elif name == "pub":
                pub.append(t - t_prev)
            elif name == "cons":
                cons.append(t - t_prev)
                t_prev = t
            elif name == "epi":
                epi.append(t - t_prev)
        if "start" in d and "end" in d and "rstart" in d and "rend" in d and d["rend"] > d["rstart"]:
            span.append(d["end"] - d["start"])
            mhz.append((d["end"] - d["start"]) / (d["rend"] - d["rstart"]) * 100.0)
            tstart.append(d["rstart"])
            tend.append(d["rend"])
    def s(x):
        return f"{st.mean(x):8.0f} (med {st.median(x):7.0f}, n {len(x)})" if x else "       -"
    print(f"workgroups {len(wgs)}, segments {len(segs)} ({sum(segs)} k-tiles)")
    if mhz:
        print(f"clock MHz            {st.median(mhz):8.0f} (p10 {sorted(mhz)[len(mhz) // 10]:.0f}, p90 {sorted(mhz)[9 * len(mhz) // 10]:.0f})")
        t0 = min(tstart)
        lat = [(e - t0) / 100.0 for e in tend]
        print(f"launch (realtime) us {max(lat):8.2f}; workgroup end times: min {min(lat):.2f} med {st.median(lat):.2f}")
        print(f"workgroup span cyc   {s(span)}")
    print(f"main cyc / k-tile    {s(per_kt)}")
    print(f"  first segment      {s(first_kt)}")
    print(f"epilogue cyc         {s(epi)}")
    print(f"publish cyc          {s(pub)}")
    print(f"consume cyc          {s(cons)}")


def main():
    ap = parser()
    ap.add_argument("--buf", default="", help="capmi_x3p_stamps / capmi_x3_stamps (default: by variant)")
    a = ap.parse_args()
    name = a.buf or ("capmi_x3_stamps" if a.x3 else "capmi_x3p_stamps")
    run, M, N, Kd = setup(a)
    for _ in range(20):  # warm, and let the clock settle under load
        run()
    torch.cuda.synchronize()
    clear(name)
    torch.cuda.synchronize()
    run()
    torch.cuda.synchronize()
    print(f"== {a.shape} M={M} N={N} K={Kd} ({name}, lib {os.path.basename(_lib.LIB_PATH)})")
    analyse(parse(read(name)))


if __name__ == "__main__":
    main()
