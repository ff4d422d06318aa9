"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) per kernel.

    python -m dash_amd.utils.profsum DB [TOP] [--dispatches PATTERN N] [--after PATTERN]

--dispatches lists the first N dispatches whose kernel name contains PATTERN in
launch order (grid size and duration), to attribute one kernel's calls to layers.
--after lists every dispatch that follows the LAST one whose name contains
PATTERN, with its start offset and the idle gap before it: e.g. `--after gg::`
is the timeline of the final batch-1 evaluation after the last garbling kernel.
"""
from __future__ import annotations

import re
import sqlite3
import sys


def _rows(db: str):
    c = sqlite3.connect(db)
    cols = {r[1] for r in c.execute("pragma table_info(rocpd_kernel_dispatch)")}
    grid = "d.grid_size_x" if "grid_size_x" in cols else "0"
    q = f"""select k.display_name, d.start, d.end, {grid} from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol k on d.kernel_id = k.id order by d.start"""
    return c.execute(q).fetchall()


def _short(name: str) -> str:
    return re.sub(r"^void ", "", re.sub(r"\(.*", "", name))


def summarize(db: str, top: int = 40) -> str:
    agg: dict[str, list] = {}
    for name, s, e, _ in _rows(db):
        a = agg.setdefault(_short(name), [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values()) or 1.0
    lines = [f"{'kernel':60s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}"]
    for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"{k[:60]:60s} {n:7d} {ms:10.3f} {1000 * ms / n:9.1f} {100 * ms / tot:6.1f}")
    lines.append(f"{'TOTAL':60s} {sum(v[0] for v in agg.values()):7d} {tot:10.3f}")
    return "\n".join(lines)


def dispatches(db: str, pattern: str, n: int) -> str:
    out = [f"# first {n} dispatches matching {pattern!r} (launch order): grid_x, us"]
    for name, s, e, g in _rows(db):
        if pattern in name:
            out.append(f"{_short(name)[:40]:40s} {g:10d} {(e - s) / 1e3:10.1f}")
            if len(out) > n:
                break
    return "\n".join(out)


def after(db: str, pattern: str) -> str:
    rows = _rows(db)
    last = max((i for i, r in enumerate(rows) if pattern in r[0]), default=-1)
    tail = rows[last + 1:]
    if not tail:
        return f"# no dispatches after the last {pattern!r}"
    t0 = tail[0][1]
    busy = sum(e - s for _, s, e, _ in tail)
    span = tail[-1][2] - t0
    out = [f"# {len(tail)} dispatches after the last {pattern!r}: span {span / 1e3:.1f} us, "
           f"kernels busy {busy / 1e3:.1f} us ({100 * busy / max(span, 1):.0f} %)",
           f"{'kernel':44s} {'grid_x':>9s} {'start_us':>9s} {'gap_us':>7s} {'us':>8s}"]
    prev = t0
    for name, s, e, g in tail:
        out.append(f"{_short(name)[:44]:44s} {g:9d} {(s - t0) / 1e3:9.1f} {(s - prev) / 1e3:7.1f} {(e - s) / 1e3:8.1f}")
        prev = e
    return "\n".join(out)


if __name__ == "__main__":
    args = sys.argv[1:]
    extra = ""
    if "--after" in args:
        i = args.index("--after")
        extra = after(args[0], args[i + 1])
        args = args[:i] + args[i + 2:]
    if "--dispatches" in args:
        i = args.index("--dispatches")
        extra += dispatches(args[0], args[i + 1], int(args[i + 2]))
        args = args[:i]
    print(summarize(args[0], int(args[1]) if len(args) > 1 else 40))
    if extra:
        print(extra)
