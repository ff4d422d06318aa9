"""The rocprofv3 kernel-trace summariser (dash_amd/utils/profsum.py) on a synthetic rocpd database."""
import sqlite3

from dash_amd.utils import profsum


def _db(path):
    c = sqlite3.connect(path)
    c.execute("create table rocpd_info_kernel_symbol (id integer, display_name text)")
    c.execute("create table rocpd_kernel_dispatch (kernel_id integer, start integer, end integer, grid_size_x integer)")
    names = ["void dash::gg::k_emit(int)", "void dash::dev::k_conv_img2<1, true>(int)", "void dash::dev::k_mrs_chain_q<7, 2>(int)"]
    c.executemany("insert into rocpd_info_kernel_symbol values (?, ?)", list(enumerate(names)))
    # garble, eval, garble, eval (the timeline after the last gg:: dispatch: conv then chain, 5 us gap)
    rows = [(0, 0, 10_000, 256), (1, 12_000, 20_000, 64), (0, 30_000, 40_000, 256), (1, 41_000, 50_000, 64),
            (2, 55_000, 75_000, 128)]
    c.executemany("insert into rocpd_kernel_dispatch values (?, ?, ?, ?)", rows)
    c.commit()
    c.close()


def test_summary_and_after(tmp_path):
    db = str(tmp_path / "t.db")
    _db(db)
    s = profsum.summarize(db)
    assert "dash::gg::k_emit" in s and "TOTAL" in s
    tl = profsum.after(db, "gg::").splitlines()
    assert "2 dispatches" in tl[0] and "span 34.0 us" in tl[0] and "busy 29.0 us" in tl[0]
    assert tl[2].split()[-3:] == ["0.0", "0.0", "9.0"] and tl[3].split()[-3:] == ["14.0", "5.0", "20.0"]
    assert "no dispatches" in profsum.after(db, "k_mrs_chain_q")
