"""The gfx950 machine code of one kernel in a built librtmi (no GPU, no ROCm
tools): the library's .hip_fatbin section holds clang offload bundles, each
with a gfx950 code object (an ELF); the kernel's bytes are its symbol's range
in that object's .text.  bench.py hashes them to check that a committed PMC
record (profiles/pmc_*.json) was measured on the kernel it is quoted for
(VERDICT r05 item 4)."""
import hashlib
import struct

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    """{name: (offset, size, link, entsize)} of a little-endian ELF64 image."""
    (shoff,) = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, _typ, _flags, _addr, off, size, link, _info, _align, entsize = struct.unpack_from(
            "<IIQQQQIIQQ", elf, shoff + i * shentsize)
        hdrs.append((name, off, size, link, entsize))
    stroff = hdrs[shstrndx][1]
    out = {}
    for name, off, size, link, entsize in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, link, entsize, hdrs)
    return out


def gfx950_code_objects(lib_bytes):
    """Every gfx950 code object in the library's offload bundles."""
    secs = _sections(lib_bytes)
    if ".hip_fatbin" not in secs:
        return []
    off, size = secs[".hip_fatbin"][:2]
    fat = lib_bytes[off:off + size]
    out, pos = [], fat.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", fat, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            o, sz, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith("gfx950"):
                out.append(fat[pos + o:pos + o + sz])
        pos = fat.find(MAGIC, pos + 1)
    return out


def kernel_code(co, symbol_part):
    """(symbol, bytes) of the function whose symbol contains symbol_part in
    one code object, or None."""
    secs = _sections(co)
    if ".symtab" not in secs or ".text" not in secs:
        return None
    soff, ssize, link, entsize, hdrs = secs[".symtab"]
    stroff = hdrs[link][1]
    text_off = secs[".text"][0]
    # .text's load address (sh_addr) maps symbol values to file offsets
    (shoff,) = struct.unpack_from("<Q", co, 0x28)
    shentsize = struct.unpack_from("<H", co, 0x3A)[0]
    text_addr = None
    for i in range(len(hdrs)):
        _n, _t, _f, addr, off, _s, _l, _i, _a, _e = struct.unpack_from("<IIQQQQIIQQ", co, shoff + i * shentsize)
        if off == text_off:
            text_addr = addr
    for k in range(ssize // entsize):
        name, info, _other, _shndx, value, size = struct.unpack_from("<IBBHQQ", co, soff + k * entsize)
        if info & 0xF != 2 or size == 0:  # STT_FUNC with a body
            continue
        end = co.index(b"\0", stroff + name)
        sym = co[stroff + name:end].decode()
        if symbol_part in sym:
            start = text_off + (value - text_addr)
            return sym, co[start:start + size]
    return None


def kernel_sha1(lib_path, symbol_part):
    """(symbol, sha1 of its gfx950 machine code) in the library, or (None, None)."""
    with open(lib_path, "rb") as f:
        data = f.read()
    for co in gfx950_code_objects(data):
        r = kernel_code(co, symbol_part)
        if r:
            return r[0], hashlib.sha1(r[1]).hexdigest()
    return None, None
