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


def _rs(name):
    return open(os.path.join(ROOT, "overlord-hip", "src", name)).read()


def test_hipcrypto_is_a_clone_drop_in():
    """the reference's ConsensusCrypto is #[derive(Clone)] (consensus.rs:339)
    and Consensus::new clones it three times (consensus.rs:61-76); update_pubkeys is
    `async fn(&self, Vec<BlsPublicKey>)` (consensus.rs:361-363, callers :131-136, :622-629)."""
    lib = _rs("lib.rs")
    m = re.search(r"#\[derive\(([^)]*)\)\]\s*pub struct HipCrypto\s*\{(.*?)\n\}", lib, flags=re.S)
    assert m and "Clone" in m.group(1), "HipCrypto must derive Clone"
    body = m.group(2)
    # every field is shared or cheap to clone: the context behind Arc (one ovh_destroy, by the
    # last clone), never a raw Ctx a naive clone would double-free
    assert re.search(r"ctx:\s*Arc<Ctx>", body), body
    assert re.search(r"pubkeys:\s*Arc<RwLock<", body), body
    assert "impl Drop for Ctx" in lib and "impl Drop for HipCrypto" not in lib
    # update_pubkeys: async, no result, takes any ophelia PublicKey (Vec<BlsPublicKey> at the call sites)
    sig = re.search(r"pub async fn update_pubkeys<K: ophelia::PublicKey>\(&self, new_pubkeys: Vec<K>\)\s*\{", lib)
    assert sig, "update_pubkeys must keep the reference's async shape"
    assert "ovh_set_validators" in lib and "spawn_blocking" in lib
    # the reference's error variants and conversion (error.rs:20-45)
    for v in ("Other(String)", "CryptoErr(i32)", "impl From<HipCryptoError> for Box<dyn Error + Send>"):
        assert v in lib, v


def test_ingress_module_mirrors_the_python_shim():
    """The VoteIngress state machine of INTEGRATION.md section 4 as overlord-hip/src/ingress.rs:
    the message kinds of consensus.rs:210-258, the per-(height, round, kind) groups, the
    prefetch on a blocking task and the forward in arrival order; its device calls are declared
    in ffi.rs (checked against the header above)."""
    lib, ing = _rs("lib.rs"), _rs("ingress.rs")
    assert "pub mod ingress;" in lib
    for kind in ('"SignedVote"', '"SignedChoke"', '"AggregatedVote"', '"SignedProposal"'):
        assert kind in ing, kind
    for call in ("pub async fn proc_network_msg", "pub async fn poll", "pub async fn flush", "spawn_blocking",
                 "crypto.prefetch(", "crypto.vote_digests("):
        assert call in ing, call
    # the library calls behind them
    assert re.search(r"ffi::ovh_prefetch\(", lib) and re.search(r"ffi::ovh_vote_digests\(", lib)
    f = ffi_protos()
    for name in ("ovh_prefetch", "ovh_vote_digests", "ovh_set_validators", "ovh_sm3"):
        assert name in f, name
    py = open(os.path.join(ROOT, "consensus_overlord_amd", "ingress.py")).read()
    for attr in ("batches", "prefetched", "forwarded", "dropped", "unbatched"):
        assert '"%s"' % attr in py and "pub %s: u64" % attr in ing, attr


def test_cargo_dependencies_are_used_and_build_writes_out_dir():
    """build.rs generates vm_progs.inc into OUT_DIR (never the source tree) and
    reruns only on real sources; every dependency of Cargo.toml is used by the crate."""
    cargo = open(os.path.join(ROOT, "overlord-hip", "Cargo.toml")).read()
    build = open(os.path.join(ROOT, "overlord-hip", "build.rs")).read()
    src = _rs("lib.rs") + _rs("ingress.rs") + _rs("ffi.rs")
    deps = re.findall(r"^(\w[\w-]*)\s*=", cargo.split("[dependencies]", 1)[1].split("\n[", 1)[0], flags=re.M)
    assert set(deps) >= {"overlord", "bytes", "ophelia", "rlp", "tokio", "hex"}
    for d in deps:
        assert re.search(r"\b%s::" % d.replace("-", "_"), src), "unused dependency " + d
    assert 'out.join("vm_progs.inc")' in build and 'src.join("csrc/vm_progs.inc")' not in build
    assert 'format!("-I{}", out.display())' in build
    assert 'rerun-if-changed={}", src.join("csrc").display()' not in build
    hip = open(os.path.join(ROOT, "consensus_overlord_amd", "csrc", "ovhip.hip")).read()
    assert "#include <vm_progs.inc>" in hip   # found through -I (OUT_DIR or csrc), not beside the file
