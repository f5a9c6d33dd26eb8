"""GPU text codec (dsort_format_text_dev_i32 / dsort_parse_text_dev_i32) against
the oracle's codec (oracle_format_i32 / oracle_parse_i32) and the reference's own
input.txt -> output.txt.  Runs on the MI355X box only (pytest -m gpu); every call goes through
the C ABI, the oracle is only the checker."""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

INT_MIN, INT_MAX = -(2**31), 2**31 - 1
FTILE = 2048    # keys per format tile (dsort_text.hip)
PTILE = 16384   # text bytes per parse tile


def _torch():
    import torch
    return torch


def gpu_format(ctx, keys, offset=0):
    torch = _torch()
    k = torch.from_numpy(np.ascontiguousarray(keys, np.int32)).cuda()
    buf = torch.empty(12 * k.numel() + offset + 16, dtype=torch.uint8, device="cuda")
    n = ctx.format_text(k, buf[offset:])
    torch.cuda.synchronize()
    return bytes(buf[offset:offset + n].cpu().numpy())


def gpu_parse(ctx, raw, cap=None):
    torch = _torch()
    t = torch.from_numpy(np.frombuffer(raw, np.uint8).copy()).cuda() if raw else \
        torch.empty(16, dtype=torch.uint8, device="cuda")
    cap = len(raw) // 2 + 1 if cap is None else cap
    keys = torch.zeros(max(cap, 1), dtype=torch.int32, device="cuda")
    cnt = ctx.parse_text(t, len(raw), keys)
    torch.cuda.synchronize()
    return cnt, keys[:min(cnt, cap)].cpu().numpy()


def boundary_keys():
    v = [0, 1, -1, 9, 10, -9, -10, INT_MIN, INT_MAX, INT_MIN + 1, INT_MAX - 1]
    for p in range(1, 10):
        v += [10**p - 1, 10**p, -(10**p - 1), -(10**p)]
    return np.array(v, np.int64).astype(np.int32)


@pytest.mark.parametrize("n", [1, 2, 7, FTILE - 1, FTILE, FTILE + 1, 3 * FTILE + 5, 100003, 1 << 20])
@pytest.mark.parametrize("kind", ["uniform", "small", "mixed"])
def test_format_vs_oracle(gpu_ctx, oracle, n, kind):
    rng = np.random.default_rng(n * 7 + len(kind))
    if kind == "uniform":
        a = rng.integers(INT_MIN, INT_MAX, n, endpoint=True).astype(np.int32)
    elif kind == "small":
        a = rng.integers(-50, 50, n).astype(np.int32)
    else:
        b = boundary_keys()
        a = b[rng.integers(0, b.size, n)]
    assert gpu_format(gpu_ctx, a) == oracle.format(a)


@pytest.mark.parametrize("offset", [1, 3, 7, 13, 15])
def test_format_unaligned_destination(gpu_ctx, oracle, offset):
    a = np.random.default_rng(offset).integers(INT_MIN, INT_MAX, 50001).astype(np.int32)
    assert gpu_format(gpu_ctx, a, offset) == oracle.format(a)


def test_format_empty(gpu_ctx):
    assert gpu_format(gpu_ctx, np.zeros(0, np.int32)) == b""


def test_format_rejects_small_buffer(gpu_ctx, dsort_mod):
    torch = _torch()
    k = torch.zeros(100, dtype=torch.int32, device="cuda")
    buf = torch.empty(12 * 100 - 1, dtype=torch.uint8, device="cuda")
    with pytest.raises(dsort_mod.DsortError):
        gpu_ctx.format_text(k, buf)


def test_reference_output_txt_bytes(gpu_ctx, oracle):
    """The reference's input.txt, parsed and sorted on the GPU, formats to its output.txt."""
    torch = _torch()
    raw = open(os.path.join(GOLDEN, "ref_input.txt"), "rb").read()
    exp = open(os.path.join(GOLDEN, "ref_output.txt"), "rb").read()
    cnt, keys = gpu_parse(gpu_ctx, raw)
    assert np.array_equal(keys, oracle.parse(raw)) and cnt == keys.size
    t = torch.from_numpy(keys).cuda()
    gpu_ctx.sort_dev(t)
    assert gpu_format(gpu_ctx, t.cpu().numpy()) == exp


@pytest.mark.parametrize("n", [1, 5, 3000, 100003, 1 << 20])
def test_parse_roundtrip_vs_oracle(gpu_ctx, oracle, n):
    a = np.random.default_rng(n).integers(INT_MIN, INT_MAX, n, endpoint=True).astype(np.int32)
    raw = oracle.format(a)
    cnt, keys = gpu_parse(gpu_ctx, raw)
    assert cnt == n and np.array_equal(keys, a)


def _messy_text(rng, vals):
    seps = [b" ", b"\n", b"\t", b"\r\n", b"  ", b" \n\t ", b"\x0b", b"\x0c"]
    out = [seps[rng.integers(0, len(seps))] if rng.random() < 0.3 else b""]
    for v in vals:
        s = str(int(v)).encode()
        r = rng.random()
        if r < 0.1 and v >= 0:
            s = b"+" + s
        elif r < 0.2:
            s = (b"-" if v < 0 else b"") + b"0" * int(rng.integers(1, 30)) + str(abs(int(v))).encode()
        out.append(s)
        out.append(seps[rng.integers(0, len(seps))])
    if rng.random() < 0.5:
        out.pop()  # no trailing whitespace
    return b"".join(out)


@pytest.mark.parametrize("seed", range(6))
def test_parse_messy_whitespace_signs_zeros(gpu_ctx, oracle, seed):
    rng = np.random.default_rng(seed)
    vals = rng.integers(INT_MIN, INT_MAX, 20000 + seed * 7000, endpoint=True)
    raw = _messy_text(rng, vals)
    cnt, keys = gpu_parse(gpu_ctx, raw)
    exp = oracle.parse(raw)
    assert cnt == exp.size and np.array_equal(keys, exp)


def test_parse_long_tokens_across_tile_and_halo(gpu_ctx, oracle):
    """Tokens longer than the staged halo (leading zeros) straddling tile boundaries."""
    parts, pos = [], 0
    rng = np.random.default_rng(5)
    while pos < 5 * PTILE:
        z = int(rng.choice([0, 3, 70, 200]))
        tok = b"0" * z + str(int(rng.integers(0, 10**6))).encode()
        parts.append(tok)
        parts.append(b" ")
        pos += len(tok) + 1
    raw = b"".join(parts)
    cnt, keys = gpu_parse(gpu_ctx, raw)
    exp = oracle.parse(raw)
    assert cnt == exp.size and np.array_equal(keys, exp)


def test_parse_overflow_saturates_like_oracle(gpu_ctx, oracle):
    raw = b"2147483647 2147483648 -2147483648 -2147483649 4294967295 4294967296 " \
          b"99999999999999999999 -99999999999999999999 4294967297"
    cnt, keys = gpu_parse(gpu_ctx, raw)
    assert np.array_equal(keys, oracle.parse(raw)) and cnt == 9


@pytest.mark.parametrize("raw", [b"", b"   \n\t  ", b"\n"])
def test_parse_no_tokens(gpu_ctx, raw):
    cnt, _ = gpu_parse(gpu_ctx, raw)
    assert cnt == 0


def test_parse_counts_past_cap(gpu_ctx):
    raw = b" ".join(str(i).encode() for i in range(1000))
    cnt, keys = gpu_parse(gpu_ctx, raw, cap=10)
    assert cnt == 1000 and keys.tolist() == list(range(10))


@pytest.mark.parametrize("raw,pos", [(b"12a", 0), (b"1 2 -", 4), (b"1 + 3", 2), (b"abc", 0),
                                     (b"--1", 0), (b"5 1-2", 2), (b"7 8\n9x 10", 4)])
def test_parse_rejects_non_integer_token(gpu_ctx, oracle, dsort_mod, raw, pos):
    with pytest.raises(ValueError):
        oracle.parse(raw)
    with pytest.raises(dsort_mod.DsortError, match=f"byte {pos}$"):
        gpu_parse(gpu_ctx, raw)


def test_parse_error_deep_in_text_reports_first(gpu_ctx, dsort_mod):
    body = b" ".join(str(i).encode() for i in range(20000))
    raw = body + b" x1 " + body + b" y "
    with pytest.raises(dsort_mod.DsortError, match=f"byte {len(body) + 1}$"):
        gpu_parse(gpu_ctx, raw)


def test_format_parse_roundtrip_2p26(gpu_ctx):
    """Full-size property: parse(format(keys)) == keys, and the byte count is the sum of the
    %d lengths."""
    torch = _torch()
    n = 1 << 26
    k = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu_ctx.gen_uniform(k, 0x5EED2026)
    buf = torch.empty(12 * n, dtype=torch.uint8, device="cuda")
    ln = gpu_ctx.format_text(k, buf)
    a = k.cpu().numpy().astype(np.int64)
    mag = np.abs(a)
    digits = np.ones(n, np.int64)
    for p in range(1, 10):
        digits += mag >= 10**p
    assert ln == int(digits.sum() + (a < 0).sum() + n)
    back = torch.empty(n, dtype=torch.int32, device="cuda")
    cnt = gpu_ctx.parse_text(buf, ln, back)
    assert cnt == n
    assert torch.equal(back, k)


def test_host_buffer_forms_match_oracle(gpu_ctx, oracle, dsort_mod):
    """dsort_parse_text_i32 / dsort_format_text_i32: the C master's parse and output.txt write."""
    raw = open(os.path.join(GOLDEN, "ref_input.txt"), "rb").read()
    assert np.array_equal(gpu_ctx.parse_text_host(raw), oracle.parse(raw))
    a = np.random.default_rng(3).integers(INT_MIN, INT_MAX, 300001, endpoint=True).astype(np.int32)
    txt = gpu_ctx.format_text_host(a)
    assert txt == oracle.format(a)
    assert np.array_equal(gpu_ctx.parse_text_host(txt), a)
    assert gpu_ctx.format_text_host(np.zeros(0, np.int32)) == b""
    with pytest.raises(dsort_mod.DsortError, match="byte 2$"):
        gpu_ctx.parse_text_host(b"1 x")
