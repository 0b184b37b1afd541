"""Writes fishnet-style asset archives for the tests (test infrastructure only).

The layout is what /root/reference/build.rs:398-420 produces with the `ar` crate's
Builder (BSD long names "#1/<len>", the name leading the member data) or, for the
GNU variant, a "//" long-name table; the archive is then zstd-compressed with the
system libzstd.so.1 (ctypes: no Python zstd package is installed)."""
import ctypes as C


def _hdr(name_field: bytes, size: int, mode: int = 0o644) -> bytes:
    h = (name_field.ljust(16) + b"0".ljust(12) + b"0".ljust(6) + b"0".ljust(6) +
         f"{mode:o}".encode().ljust(8) + str(size).encode().ljust(10) + b"`\n")
    assert len(h) == 60
    return h


def ar_bytes(members, gnu=False) -> bytes:
    """members: [(name, data)] -> `ar` image."""
    out = [b"!<arch>\n"]
    if gnu:
        table, offs = b"", []
        for name, _ in members:
            offs.append(len(table))
            table += name.encode() + b"/\n"
        out += [_hdr(b"//", len(table)), table + (b"\n" if len(table) & 1 else b"")]
        for (name, data), o in zip(members, offs):
            nm = name.encode()
            field = nm + b"/" if len(nm) < 16 else f"/{o}".encode()
            out += [_hdr(field, len(data)), data + (b"\n" if len(data) & 1 else b"")]
    else:
        for name, data in members:
            nm = name.encode()
            if len(nm) <= 16 and b" " not in nm:
                out += [_hdr(nm, len(data)), data]
                size = len(data)
            else:
                out += [_hdr(f"#1/{len(nm)}".encode(), len(nm) + len(data)), nm + data]
                size = len(nm) + len(data)
            if size & 1:
                out.append(b"\n")
    return b"".join(out)


def zstd(data: bytes, level: int = 3) -> bytes:
    z = C.CDLL("libzstd.so.1")
    z.ZSTD_compressBound.restype = C.c_size_t
    z.ZSTD_compressBound.argtypes = [C.c_size_t]
    z.ZSTD_compress.restype = C.c_size_t
    z.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    z.ZSTD_isError.argtypes = [C.c_size_t]
    cap = z.ZSTD_compressBound(len(data))
    dst = C.create_string_buffer(cap)
    n = z.ZSTD_compress(dst, cap, data, len(data), level)
    assert not z.ZSTD_isError(n)
    return dst.raw[:n]
