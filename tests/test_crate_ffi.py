"""The overlord-hip crate's FFI (overlord-hip/src/ffi.rs) against the C ABI (include/ovhip.h).

There is no Rust toolchain in this image, so the crate is not compiled here; this test keeps
its `extern "C"` block in sync with the header mechanically: every prototype of the header has
exactly one declaration in ffi.rs with the same name, the same argument count and order, and
the Rust type the C type maps to (int -> i32, size_t -> usize, uintN_t -> uN, int32_t -> i32,
float -> f32, `const T*` -> `*const T`, `T*` / `T out[k]` -> `*mut T`), and the same return type;
the crate's error constants equal the header's. The trait surface it implements is the
reference's `Crypto` impl (consensus.rs:385-463): the five method names are checked in lib.rs.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "ovhip.h")
FFI = os.path.join(ROOT, "overlord-hip", "src", "ffi.rs")
LIB = os.path.join(ROOT, "overlord-hip", "src", "lib.rs")

C2R = {"int": "i32", "size_t": "usize", "uint32_t": "u32", "uint64_t": "u64", "uint8_t": "u8", "int32_t": "i32",
       "float": "f32", "char": "c_char", "void": "c_void", "ovh_ctx": "OvhCtx"}


def c_type(t: str) -> str:
    t = " ".join(t.split())
    const = t.startswith("const ")
    if const:
        t = t[len("const "):]
    if t.endswith("*"):
        return ("*const " if const else "*mut ") + C2R[t[:-1].strip()]
    return C2R[t]


def header_protos():
    h = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    out = {}
    for m in re.finditer(r"^(ovh_ctx\*|int|void\*|void|const char\*) (ovh_\w+)\(([^;]*)\);", h, flags=re.M):
        ret, name, args = m.groups()
        types = []
        for a in [x.strip() for x in " ".join(args.split()).split(",") if x.strip()]:
            am = re.match(r"(.*?)(\w+)(\[\d+\])?$", a)
            ty, _, arr = am.groups()
            types.append(c_type(ty.strip() + ("*" if arr else "")))
        out[name] = (types, None if ret == "void" else c_type(ret))
    return out


def ffi_protos():
    s = open(FFI).read()
    blk = s[s.index('extern "C" {'):]
    out = {}
    for m in re.finditer(r"pub fn (ovh_\w+)\((.*?)\)(?:\s*->\s*([^;]+))?;", blk, flags=re.S):
        name, args, ret = m.groups()
        types = [a.split(":", 1)[1].strip() for a in [x.strip() for x in " ".join(args.split()).split(",")] if a]
        assert name not in out, "duplicate declaration of %s" % name
        out[name] = (types, ret.strip() if ret else None)
    return out


def test_every_header_prototype_is_declared_identically():
    h, f = header_protos(), ffi_protos()
    assert len(h) >= 40
    assert set(h) == set(f), (sorted(set(h) - set(f)), sorted(set(f) - set(h)))
    for name in h:
        assert h[name] == f[name], (name, h[name], f[name])


def test_constants_match_the_header():
    hdr = open(HDR).read()
    ffi = open(FFI).read()
    for m in re.finditer(r"#define (OVH_(?:OK|ERR_\w+|FLAG_\w+|NSTAGES|VOTE_HASH_MAX|PARTIAL_BYTES|BATCH_SLOTS)) "
                         r"(0x[0-9a-f]+u?|\d+)", hdr):
        name, val = m.group(1), int(m.group(2).rstrip("u"), 0)
        r = re.search(r"pub const %s: \w+ = (0x[0-9a-f]+|\d+);" % name, ffi)
        assert r, name
        assert int(r.group(1), 0) == val, name


def test_crypto_trait_methods_and_build_script():
    lib = open(LIB).read()
    for fn in ("fn hash(", "fn sign(", "fn verify_signature(", "fn aggregate_signatures(",
               "fn verify_aggregated_signature("):
        assert fn in lib, fn
    # the reference's error strings (consensus.rs:391-462)
    for msg in ("failed to convert hash value", "signatures length does not match voters length", "lose public key"):
        assert msg in lib, msg
    build = open(os.path.join(ROOT, "overlord-hip", "build.rs")).read()
    assert "--offload-arch={arch}" in build and '"gfx950"' in build and "gen.py" in build
