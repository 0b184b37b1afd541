// archive.h — reading a net out of fishnet's asset archive (host code of libgpu_nnue).
//
// fishnet bundles its engines and both .nnue files in one zstd-compressed `ar`
// archive, assets.ar.zst: build.rs appends every file with `ar::Builder`
// (/root/reference/build.rs:398-420) and Assets::prepare streams it back through a
// ZstdDecoder into `ar::Archive` (/root/reference/src/assets.rs:186-226).  This is
// the same two layers, restated:
//   zstd  — decompressed with the system libzstd (libzstd.so.1, opened at run time:
//           no build dependency; a plain, uncompressed `ar` is accepted as well);
//   ar    — "!<arch>\n", then per member a 60-byte header (name[16] mtime[12]
//           uid[6] gid[6] mode[8] size[10] "`\n") and the data padded to an even
//           length.  Long names: BSD "#1/<len>" (the name is the first <len> bytes
//           of the data, as the `ar` crate's Builder writes them) and GNU "/<offset>"
//           into the "//" table; short GNU names end in '/'.
#pragma once
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

namespace gn {
namespace archive {

struct ZBufIn {
  const void *src;
  size_t size, pos;
};
struct ZBufOut {
  void *dst;
  size_t size, pos;
};

// Decompresses every frame of a zstd stream.  Returns false with a message.
inline bool zstd_decompress(const uint8_t *src, size_t n, std::vector<uint8_t> &out, std::string &err) {
  void *h = dlopen("libzstd.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    err = "libzstd.so.1 not found (needed for .zst archives)";
    return false;
  }
  typedef void *(*create_t)();
  typedef size_t (*init_t)(void *);
  typedef size_t (*step_t)(void *, ZBufOut *, ZBufIn *);
  typedef size_t (*free_t)(void *);
  typedef unsigned (*iserr_t)(size_t);
  typedef const char *(*name_t)(size_t);
  auto create = (create_t)dlsym(h, "ZSTD_createDStream");
  auto init = (init_t)dlsym(h, "ZSTD_initDStream");
  auto step = (step_t)dlsym(h, "ZSTD_decompressStream");
  auto fr = (free_t)dlsym(h, "ZSTD_freeDStream");
  auto iserr = (iserr_t)dlsym(h, "ZSTD_isError");
  auto ename = (name_t)dlsym(h, "ZSTD_getErrorName");
  if (!create || !init || !step || !fr || !iserr || !ename) {
    err = "libzstd.so.1 lacks the streaming decompression API";
    dlclose(h);
    return false;
  }
  void *ds = create();
  bool ok = ds != nullptr && !iserr(init(ds));
  ZBufIn in = {src, n, 0};
  std::vector<uint8_t> chunk(1 << 20);
  size_t last = 0;
  while (ok && in.pos < in.size) {
    ZBufOut o = {chunk.data(), chunk.size(), 0};
    last = step(ds, &o, &in);
    if (iserr(last)) {
      err = std::string("zstd: ") + ename(last);
      ok = false;
      break;
    }
    out.insert(out.end(), chunk.data(), chunk.data() + o.pos);
    if (o.pos == 0 && in.pos == in.size) break;
  }
  while (ok && last != 0) { // flush what the decoder still holds
    ZBufOut o = {chunk.data(), chunk.size(), 0};
    last = step(ds, &o, &in);
    if (iserr(last)) {
      err = std::string("zstd: ") + ename(last);
      ok = false;
      break;
    }
    out.insert(out.end(), chunk.data(), chunk.data() + o.pos);
    if (o.pos == 0) {
      if (last != 0) err = "zstd: truncated stream", ok = false;
      break;
    }
  }
  if (ds) fr(ds);
  dlclose(h);
  return ok;
}

struct Member {
  std::string name;
  size_t off, size; // data bytes within the archive image
};

inline bool parse_decimal(const uint8_t *p, int len, size_t &v) {
  v = 0;
  int i = 0;
  while (i < len && p[i] == ' ') ++i;
  if (i == len || p[i] < '0' || p[i] > '9') return false;
  for (; i < len && p[i] >= '0' && p[i] <= '9'; ++i) v = v * 10 + (size_t)(p[i] - '0');
  for (; i < len; ++i)
    if (p[i] != ' ') return false;
  return true;
}

// The members of an `ar` image (names resolved, GNU symbol / name tables skipped).
inline bool ar_members(const uint8_t *a, size_t n, std::vector<Member> &out, std::string &err) {
  if (n < 8 || memcmp(a, "!<arch>\n", 8) != 0) {
    err = "not an ar archive";
    return false;
  }
  size_t p = 8;
  const uint8_t *gnu_names = nullptr;
  size_t gnu_len = 0;
  while (p < n) {
    if (p + 60 > n || a[p + 58] != '`' || a[p + 59] != '\n') {
      err = "truncated or corrupt ar member header";
      return false;
    }
    size_t size;
    if (!parse_decimal(a + p + 48, 10, size) || p + 60 + size > n) {
      err = "bad ar member size";
      return false;
    }
    const uint8_t *h = a + p;
    size_t doff = p + 60, dsize = size;
    std::string name;
    if (h[0] == '#' && h[1] == '1' && h[2] == '/') { // BSD long name, stored in the data
      size_t nl;
      if (!parse_decimal(h + 3, 13, nl) || nl > size) {
        err = "bad BSD long name";
        return false;
      }
      name.assign((const char *)a + doff, nl);
      name = name.c_str(); // the crate may pad with NULs
      doff += nl, dsize -= nl;
    } else if (h[0] == '/' && h[1] == '/') { // GNU long-name table
      gnu_names = a + doff, gnu_len = size;
      name.clear();
    } else if (h[0] == '/' && (h[1] == ' ' || h[1] == '\0')) { // GNU symbol table
      name.clear();
    } else if (h[0] == '/') { // GNU "/<offset>" into the name table
      size_t o;
      if (!gnu_names || !parse_decimal(h + 1, 15, o) || o >= gnu_len) {
        err = "bad GNU long-name reference";
        return false;
      }
      size_t e = o;
      while (e < gnu_len && gnu_names[e] != '/' && gnu_names[e] != '\n') ++e;
      name.assign((const char *)gnu_names + o, e - o);
    } else {
      int e = 16;
      while (e > 0 && h[e - 1] == ' ') --e;
      if (e > 0 && h[e - 1] == '/') --e; // GNU short-name terminator
      name.assign((const char *)h, (size_t)e);
    }
    if (!name.empty()) out.push_back({name, doff, dsize});
    p += 60 + size + (size & 1);
  }
  return true;
}

// The image of an archive file: zstd-decompressed when it starts with the zstd magic.
inline bool load_image(const std::vector<uint8_t> &file, std::vector<uint8_t> &img, std::string &err) {
  static const uint8_t ZMAGIC[4] = {0x28, 0xB5, 0x2F, 0xFD};
  if (file.size() >= 4 && memcmp(file.data(), ZMAGIC, 4) == 0) return zstd_decompress(file.data(), file.size(), img, err);
  img = file;
  return true;
}

} // namespace archive
} // namespace gn
