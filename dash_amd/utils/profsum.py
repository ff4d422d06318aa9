"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite) per kernel."""
from __future__ import annotations

import re
import sqlite3
import sys


def summarize(db: str, top: int = 40) -> str:
    c = sqlite3.connect(db)
    q = """select k.display_name, d.start, d.end from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol k on d.kernel_id = k.id"""
    rows = c.execute(q).fetchall()
    agg: dict[str, list] = {}
    for name, s, e in rows:
        short = re.sub(r"\(.*", "", name)
        short = re.sub(r"^void ", "", short)
        a = agg.setdefault(short, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e6
    tot = sum(v[1] for v in agg.values()) or 1.0
    lines = [f"{'kernel':60s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}"]
    for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        lines.append(f"{k[:60]:60s} {n:7d} {ms:10.3f} {1000 * ms / n:9.1f} {100 * ms / tot:6.1f}")
    lines.append(f"{'TOTAL':60s} {sum(v[0] for v in agg.values()):7d} {tot:10.3f}")
    return "\n".join(lines)


if __name__ == "__main__":
    print(summarize(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 40))
