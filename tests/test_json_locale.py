"""The rapidjson::Value overloads of include/octvr.hpp (the reference callers' entry points,
octvr.hpp:75-84; apps/octvr/dump.cpp:71-96) under a comma-decimal locale: the reference's
caller is a Qt application, and Qt calls setlocale(LC_ALL, ""), so printf / strtod would write and
read 1.5 as "1,5".  The C++ layer serialises with std::to_chars and the library parses with
std::from_chars (OCTVR_JSON_EXACT), both locale-independent.

lib/vr_dump_rj (tests/cpp/vr_dump_rj.cpp, dump.cpp's flow) is compiled by build() against rapidjson's
headers where they exist; `-s` stops after the template constructor, which needs no GPU.  The
comma locale is compiled here with localedef from a minimal source (the image ships no locale data)."""
import math
import os
import shutil
import subprocess

import pytest

import oracle_py as O

BIN = os.path.join(O.ROOT, "opencv-octvr_amd", "lib", "vr_dump_rj")


def comma_locale(tmp):
    """(env additions) activating a locale whose LC_NUMERIC decimal point is ',', or None."""
    if not shutil.which("localedef"):
        return None
    cm = ["<code_set_name> ANSI_X3.4-1968", "<comment_char> %", "<escape_char> /", "CHARMAP"]
    cm += ["<U%04X> /x%02x" % (c, c) for c in range(128)] + ["END CHARMAP"]
    (tmp / "ascii.cm").write_text("\n".join(cm) + "\n")
    (tmp / "comma.src").write_text('comment_char %\nescape_char /\nLC_CTYPE\nEND LC_CTYPE\nLC_NUMERIC\n'
                                   'decimal_point "<U002C>"\nthousands_sep "<U002E>"\ngrouping 3;3\nEND LC_NUMERIC\n')
    subprocess.run(["localedef", "-c", "-f", str(tmp / "ascii.cm"), "-i", str(tmp / "comma.src"), str(tmp / "xx_XX")],
                   capture_output=True)
    if not (tmp / "xx_XX" / "LC_NUMERIC").exists():
        return None
    return {"LOCPATH": str(tmp), "LC_ALL": "xx_XX"}


def _size(cfg_path, env):
    r = subprocess.run([BIN, "-s", "-w", "1000", str(cfg_path)], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr
    return r.stdout.split()


@pytest.mark.skipif(not os.path.exists(BIN), reason="vr_dump_rj is built only where rapidjson's headers exist")
def test_rapidjson_overloads_under_comma_locale(tmp_path):
    env = comma_locale(tmp_path)
    if env is None:
        pytest.skip("localedef could not build a comma-decimal locale")
    # equirectangular output, height derived from the aspect ratio (template.cpp:23-44,
    # equirectangular.hpp:26-34): min_lat / max_lat travel through json_exact
    lo, hi = -0.78539816339744828, 1.2345678901234567
    cfg = tmp_path / "cfg.json"
    cfg.write_text('{"output": {"type": "equirectangular", "options": {"min_lat": %r, "max_lat": %r}}, "inputs": []}'
                   % (lo, hi))
    w, h, g = _size(cfg, env)
    assert g == "1,5", "the comma locale is not active in the caller"
    wc, hc, gc = _size(cfg, {"LC_ALL": "C"})
    assert gc == "1.5"
    # same size in both locales, and the one the doubles give (aspect = 2 / ((max - min) / pi))
    assert (w, h) == (wc, hc)
    assert int(w) == 1000 and int(h) == int(1000.0 / (2.0 / ((hi - lo) / math.pi)))


@pytest.mark.skipif(not os.path.exists(BIN), reason="vr_dump_rj is built only where rapidjson's headers exist")
def test_rapidjson_overloads_exact_doubles(tmp_path):
    """Doubles whose shortest form needs 17 digits, and ones rapidjson 1.0.2 parses differently from a
    correctly rounded parse, arrive unchanged: the height the library derives equals the one the
    caller's own doubles give."""
    for lo, hi in [(-0.1, 0.30000000000000004), (-1.5707963267948966, 1.5707963267948963), (-1e-7, 2.2250738585072014e-3)]:
        cfg = tmp_path / "c.json"
        cfg.write_text('{"output": {"type": "equirectangular", "options": {"min_lat": %r, "max_lat": %r}}}' % (lo, hi))
        w, h, _ = _size(cfg, {"LC_ALL": "C"})
        lo_rj, hi_rj = (O.json_loads_rj(repr(v)) for v in (lo, hi))  # the doubles the caller's rapidjson holds
        assert int(h) == int(1000.0 / (2.0 / ((hi_rj - lo_rj) / math.pi))), (lo, hi)


@pytest.mark.parametrize("text,want", [
    ("4.9e-324", 5e-324),                 # the smallest subnormal
    ("2.2250738585072011e-308", 2.2250738585072011e-308),  # below DBL_MIN: subnormal
    ("1e-400", 0.0),                      # underflow to 0, as strtod
    ("-1e-400", -0.0),
    ("1e400", math.inf),                  # overflow to HUGE_VAL, as strtod
    ("[-1.7976931348623159e308]", -math.inf),
    ("0.30000000000000004", 0.30000000000000004),
])
def test_exact_numbers_out_of_range_as_strtod(product_lib, text, want):
    """OCTVR_JSON_EXACT parsing (std::from_chars) keeps strtod's answer for literals outside the normal
    double range: overflow gives +-HUGE_VAL, underflow the subnormal or 0, instead of a
    parse error (some libstdc++ versions report result_out_of_range for subnormals)."""
    got = product_lib.debug_json_number(text, exact=True)
    assert got == want and math.copysign(1.0, got) == math.copysign(1.0, want)
