"""Symbolises scripts/pmu_sample.py histograms: ip -> (object, function) via the recorded
/proc/self/maps, the objects' ELF load segments and `nm` (symtab, else dynsym). Run where the
same object files exist (the .so files built here travel to the box unchanged; system
libraries are the same image). Prints per configuration the top functions by share of samples
and, for pairs of configurations, the per-poll sample counts side by side.

Usage: python scripts/pmu_symbolize.py gpurun_out/pmu_sample [top]"""
import bisect
import collections
import json
import os
import struct
import subprocess
import sys


def load_segments(path):
    with open(path, "rb") as f:
        h = f.read(64)
        if h[:4] != b"\x7fELF" or h[4] != 2:
            return []
        phoff, = struct.unpack_from("<Q", h, 32)
        phentsize, phnum = struct.unpack_from("<HH", h, 54)
        f.seek(phoff)
        ph = f.read(phentsize * phnum)
    segs = []
    for i in range(phnum):
        p_type, _flags, p_offset, p_vaddr, _paddr, p_filesz = struct.unpack_from("<IIQQQQ", ph, i * phentsize)
        if p_type == 1:
            segs.append((p_offset, p_vaddr, p_filesz))
    return segs


_syms = {}


def symbols(path):
    if path in _syms:
        return _syms[path]
    out = []
    for args in (["nm", "-C", "--defined-only", path], ["nm", "-D", "-C", "--defined-only", path]):
        try:
            r = subprocess.run(args, capture_output=True, text=True, timeout=60)
        except (OSError, subprocess.TimeoutExpired):
            continue
        for line in r.stdout.splitlines():
            parts = line.split(" ", 2)
            if len(parts) == 3 and parts[1] in "tTwWiI":
                try:
                    out.append((int(parts[0], 16), parts[2]))
                except ValueError:
                    pass
        if out:
            break
    out.sort()
    _syms[path] = ([a for a, _ in out], [n for _, n in out])
    return _syms[path]


def parse_maps(text):
    maps = []
    for line in text.splitlines():
        parts = line.split()
        if len(parts) < 6:
            continue
        lo, hi = (int(x, 16) for x in parts[0].split("-"))
        maps.append((lo, hi, int(parts[2], 16), parts[5]))
    maps.sort()
    return maps


def symbolise(ip, maps):
    i = bisect.bisect_right([m[0] for m in maps], ip) - 1
    if i < 0 or ip >= maps[i][1]:
        return "?", "?"
    lo, _hi, off, path = maps[i]
    file_off = ip - lo + off
    name = os.path.basename(path)
    if not os.path.exists(path):
        # the box's checkout path: map it onto this tree
        tail = path.split("/kube_sqs_autoscaler_amd/", 1)
        local = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "kube_sqs_autoscaler_amd",
                             tail[1]) if len(tail) == 2 else path
        if not os.path.exists(local):
            return name, f"+{file_off:#x}"
        path = local
    vaddr = file_off
    for p_off, p_vaddr, p_filesz in load_segments(path):
        if p_off <= file_off < p_off + p_filesz:
            vaddr = file_off - p_off + p_vaddr
            break
    addrs, names = symbols(path)
    j = bisect.bisect_right(addrs, vaddr) - 1
    return name, (names[j] if j >= 0 else f"+{vaddr:#x}")


def profile(fname):
    d = json.load(open(fname))
    maps = parse_maps(d["maps"])
    by_fn = collections.Counter()
    for ip, n in d["hist"].items():
        obj, fn = symbolise(int(ip, 16), maps)
        by_fn[f"{obj}: {fn}"] += n
    return d, by_fn


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmu_sample"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 25
    profiles = {}
    for f in sorted(os.listdir(root)):
        if f.endswith(".json"):
            d, by_fn = profile(os.path.join(root, f))
            profiles[(d["event"], f'{d["queues"]}{"tls" if d.get("tls") else ""}')] = (d, by_fn)
    for event in sorted({e for e, _ in profiles}):
        qs = sorted(q for e, q in profiles if e == event)
        print(f"== {event}: samples x period per poll, by function ({', '.join(f'q{q}' for q in qs)}) ==")
        rows = collections.Counter()
        per_poll = {}
        for q in qs:
            d, by_fn = profiles[(event, q)]
            scale = d["period"] / d["polls"]
            per_poll[q] = {k: v * scale for k, v in by_fn.items()}
            for k, v in per_poll[q].items():
                rows[k] = max(rows[k], v)
            print(f"   q{q}: p50 {d['p50_ms']} ms, {d['samples']} samples, lost {d['lost']}, "
                  f"total {sum(per_poll[q].values()):.0f} per poll")
        for k, _ in rows.most_common(top):
            print("  " + "  ".join(f"{per_poll[q].get(k, 0):10.1f}" for q in qs) + f"  {k[:150]}")


if __name__ == "__main__":
    main()
