"""The cgo binding in INTEGRATION.md (§8 f4) cannot be compiled here (no Go toolchain), so this checks it
against the C ABI it binds: every C.gsv_* function it calls is declared in include/gsv.h and exported
by libgsv.so's build, with the declared number of arguments, and every C.GSV_* constant it names is
defined there."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _go_blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```go\n(.*?)```", text, re.S)


def _prototypes():
    h = open(os.path.join(ROOT, "include", "gsv.h")).read()
    h = re.sub(r"/\*.*?\*/", "", h, flags=re.S)
    protos = {}
    for m in re.finditer(r"\b(gsv_\w+)\s*\(([^;{]*?)\)\s*;", h):
        params = m.group(2).strip()
        protos[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    consts = set(re.findall(r"#define\s+(GSV_\w+)", h)) | set(re.findall(r"\b(GSV_\w+)\s*=", h))
    return protos, consts


def _calls(code):
    """(name, number of top-level arguments) of every C.gsv_*( ... ) call"""
    out = []
    for m in re.finditer(r"\bC\.(gsv_\w+)\(", code):
        depth, i, args, cur = 1, m.end(), 0, ""
        while depth:
            ch = code[i]
            if ch in "([{":
                depth += 1
            elif ch in ")]}":
                depth -= 1
            if depth == 1 and ch == ",":
                args += 1
                cur = ""
            elif depth >= 1:
                cur += ch
            i += 1
        nargs = 0 if code[m.end():i - 1].strip() == "" else args + 1
        out.append((m.group(1), nargs))
    return out


def test_binding_calls_declared_functions_with_declared_arity():
    protos, _ = _prototypes()
    calls = [c for b in _go_blocks() for c in _calls(b)]
    assert len(calls) > 20  # the binding covers every batch entry point
    bad = [(n, a, protos.get(n)) for n, a in calls if protos.get(n) != a]
    assert not bad, bad


def test_binding_constants_are_defined():
    _, consts = _prototypes()
    used = set(re.findall(r"\bC\.(GSV_\w+)", "".join(_go_blocks())))
    assert used and not (used - consts), sorted(used - consts)


def test_binding_covers_the_batch_entry_points():
    protos, _ = _prototypes()
    called = {n for b in _go_blocks() for n, _ in _calls(b)}
    # the entry points a Go caller needs for §8's rows (the _dev forms take device pointers a Go
    # process gets from its own HIP allocation, bound the same way)
    for name in ("gsv_ecrecover_batch", "gsv_keccak256_batch", "gsv_sender_batch", "gsv_bn256_pairing_check_batch",
                 "gsv_chunk_root_batch", "gsv_notary_validate_shards", "gsv_notary_validate_partition",
                 "gsv_comm_init", "gsv_comm_unique_id"):
        assert name in protos, name
        assert name in called, name
