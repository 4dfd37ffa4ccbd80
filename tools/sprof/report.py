"""PROFILING INFRASTRUCTURE ONLY: attribute tools/sprof/sprof.c samples to
functions (addr2line -f -C on each mapped file), print the top entries.

    python tools/sprof/report.py SAMPLES [TOP] [FILTER]"""
import collections
import subprocess
import sys


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    filt = sys.argv[3] if len(sys.argv) > 3 else None
    maps, pcs, stacks = [], [], []
    for line in open(path):
        if line.startswith("M "):
            f = line[2:].split()
            if len(f) >= 6 and "x" in f[1]:
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                maps.append((lo, hi, int(f[2], 16), f[5]))
        else:
            st = [int(x, 16) for x in line.split()]
            pcs.append(st[0])
            stacks.append(st)
    byfile = collections.defaultdict(list)
    other = 0
    for pc in pcs:
        for lo, hi, off, name in maps:
            if lo <= pc < hi:
                byfile[name].append(pc - lo + off)
                break
        else:
            other += 1
    counts = collections.Counter()
    for name, offs in byfile.items():
        if filt and filt not in name:
            counts["[%s]" % name.split("/")[-1]] += len(offs)
            continue
        uniq = sorted(set(offs))
        p = subprocess.run(["addr2line", "-f", "-C", "-e", name] + ["%x" % o for o in uniq],
                           capture_output=True, text=True)
        lines = p.stdout.splitlines()
        fn = {o: lines[2 * i] for i, o in enumerate(uniq)} if len(lines) == 2 * len(uniq) else {}
        if all(v == "??" for v in fn.values()):  # no debug info: the nearest dynamic symbol
            syms = []
            for ln in subprocess.run(["nm", "-D", "--defined-only", name], capture_output=True,
                                     text=True).stdout.splitlines():
                f = ln.split()
                if len(f) == 3 and f[1] in "TtWi":
                    syms.append((int(f[0], 16), f[2]))
            syms.sort()
            import bisect
            keys = [a for a, _ in syms]
            fn = {o: (syms[bisect.bisect_right(keys, o) - 1][1] if bisect.bisect_right(keys, o) else "?")
                  for o in uniq}
        for o in offs:
            counts[fn.get(o, "?")[:110] + "  [" + name.split("/")[-1] + "]"] += 1
    tot = len(pcs)
    print("%d samples (%d unmapped)" % (tot, other))
    for k, v in counts.most_common(top):
        print("%6.2f%%  %s" % (100.0 * v / tot, k))


if __name__ == "__main__" and "--callers" not in sys.argv:
    main()


def callers(path, leaf_file, in_file, top=30):
    """Samples whose PC lies in `leaf_file`, by their first caller frame in `in_file`."""
    maps, stacks = [], []
    for line in open(path):
        if line.startswith("M "):
            f = line[2:].split()
            if len(f) >= 6 and "x" in f[1]:
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                maps.append((lo, hi, int(f[2], 16), f[5]))
        else:
            stacks.append([int(x, 16) for x in line.split()])

    def where(pc):
        for lo, hi, off, name in maps:
            if lo <= pc < hi:
                return name, pc - lo + off
        return None, 0
    offs = []
    for st in stacks:
        n, _ = where(st[0])
        if not n or leaf_file not in n:
            continue
        for pc in st[1:]:
            n2, o2 = where(pc)
            if n2 and in_file in n2:
                offs.append((n2, o2 - 1))
                break
        else:
            offs.append(("?", 0))
    c = collections.Counter()
    for name in set(n for n, _ in offs if n != "?"):
        uniq = sorted(set(o for n, o in offs if n == name))
        out = subprocess.run(["addr2line", "-f", "-C", "-i", "-e", name] + ["%x" % o for o in uniq],
                             capture_output=True, text=True).stdout.splitlines()
        p = subprocess.run(["addr2line", "-C", "-e", name] + ["%x" % o for o in uniq], capture_output=True,
                           text=True).stdout.splitlines()
        fn = subprocess.run(["addr2line", "-f", "-C", "-e", name] + ["%x" % o for o in uniq],
                            capture_output=True, text=True).stdout.splitlines()
        m = {o: fn[2 * i][:60] + " " + p[i].split("/")[-1] for i, o in enumerate(uniq)}
        for n, o in offs:
            if n == name:
                c[m[o]] += 1
    c["?"] = sum(1 for n, _ in offs if n == "?")
    tot = len(stacks)
    for k, v in c.most_common(top):
        print("%6.2f%%  %s" % (100.0 * v / tot, k))


if __name__ == "__main__" and len(sys.argv) > 4 and sys.argv[4] == "--callers":
    callers(sys.argv[1], sys.argv[2], sys.argv[3])
