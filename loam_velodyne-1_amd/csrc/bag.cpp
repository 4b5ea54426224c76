// Recorded-sweep ingest (include/loam/loam_bag.h): a rosbag v2.0 reader and the ROS1 wire formats
// of sensor_msgs/PointCloud2 and sensor_msgs/Imu, host only.  Replaces the ROS topic plumbing
// that delivers /velodyne_points and /imu/data to the reference's callbacks
// (src/scanRegistration.cpp:211-226, :638-660) when a bag is replayed.
//
// rosbag v2.0: "#ROSBAG V2.0\n", then records = u32 header_len, header (u32 field_len,
// "name=value" fields), u32 data_len, data.  op (header field) 0x03 bag header, 0x05 chunk
// (fields compression "none" / "bz2" / "lz4", size = uncompressed bytes; data = records), 0x07
// connection (conn, topic; data = the connection header with type, md5sum, ...), 0x02 message
// data (conn, time = u32 sec + u32 nsec), 0x04 index data, 0x06 chunk info.  Messages are yielded
// in file order, which is what `rosbag play` publishes for chunked bags written by
// `rosbag record`.
#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/loam/loam_bag.h"
#include "engine.hpp"

namespace {

using loam::set_last_error;

int bag_fail(int code, const std::string& m) {
  set_last_error(m);
  return code;
}

uint32_t rd_u32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

// header fields of one record: name -> (pointer, length) into the record
struct Fields {
  std::map<std::string, std::pair<const uint8_t*, uint32_t>> f;
  bool parse(const uint8_t* p, uint32_t n) {
    uint32_t i = 0;
    while (i < n) {
      if (n - i < 4) return false;
      const uint32_t len = rd_u32(p + i);
      i += 4;
      if (len > n - i) return false;
      const uint8_t* q = p + i;
      const uint8_t* eq = (const uint8_t*)std::memchr(q, '=', len);
      if (!eq) return false;
      f[std::string((const char*)q, eq - q)] = {eq + 1, (uint32_t)(len - (eq - q) - 1)};
      i += len;
    }
    return true;
  }
  bool has(const char* k) const { return f.count(k) != 0; }
  std::string str(const char* k) const {
    auto it = f.find(k);
    return it == f.end() ? std::string() : std::string((const char*)it->second.first, it->second.second);
  }
  bool u8(const char* k, uint8_t& v) const {
    auto it = f.find(k);
    if (it == f.end() || it->second.second < 1) return false;
    v = it->second.first[0];
    return true;
  }
  bool u32(const char* k, uint32_t& v) const {
    auto it = f.find(k);
    if (it == f.end() || it->second.second < 4) return false;
    v = rd_u32(it->second.first);
    return true;
  }
};

// the system compression libraries, loaded on first use (no headers needed: the two entry points
// of each are declared here with their documented signatures)
struct Codecs {
  void* bz2 = nullptr;
  void* lz4 = nullptr;
  int (*bz_decompress)(char*, unsigned*, char*, unsigned, int, int) = nullptr;
  size_t (*lz4f_create)(void**, unsigned) = nullptr;
  size_t (*lz4f_free)(void*) = nullptr;
  size_t (*lz4f_decompress)(void*, void*, size_t*, const void*, size_t*, const void*) = nullptr;
  unsigned (*lz4f_iserror)(size_t) = nullptr;
  bool load_bz2() {
    if (bz_decompress) return true;
    if (!bz2) bz2 = dlopen("libbz2.so.1", RTLD_NOW | RTLD_LOCAL);
    if (bz2) bz_decompress = (int (*)(char*, unsigned*, char*, unsigned, int, int))dlsym(bz2, "BZ2_bzBuffToBuffDecompress");
    return bz_decompress != nullptr;
  }
  bool load_lz4() {
    if (lz4f_decompress) return true;
    if (!lz4) lz4 = dlopen("liblz4.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!lz4) return false;
    lz4f_create = (size_t (*)(void**, unsigned))dlsym(lz4, "LZ4F_createDecompressionContext");
    lz4f_free = (size_t (*)(void*))dlsym(lz4, "LZ4F_freeDecompressionContext");
    lz4f_decompress = (size_t (*)(void*, void*, size_t*, const void*, size_t*, const void*))dlsym(lz4, "LZ4F_decompress");
    lz4f_iserror = (unsigned (*)(size_t))dlsym(lz4, "LZ4F_isError");
    if (!lz4f_create || !lz4f_free || !lz4f_iserror) lz4f_decompress = nullptr;
    return lz4f_decompress != nullptr;
  }
};
Codecs g_codecs;

}  // namespace

struct loam_bag {
  FILE* f = nullptr;
  std::vector<uint8_t> chunk;   // decompressed records of the current chunk
  size_t chunk_pos = 0;
  std::vector<uint8_t> rec_hdr, rec_data;
  std::map<uint32_t, std::pair<std::string, std::string>> conns;  // conn -> (topic, type)
  std::vector<uint8_t> msg;     // the message handed out by loam_bag_next
};

namespace {

// one record from the file (false at a clean end of file)
int read_record(loam_bag* b, std::vector<uint8_t>& hdr, std::vector<uint8_t>& data) {
  uint8_t len4[4];
  const size_t got = std::fread(len4, 1, 4, b->f);
  if (got == 0) return LOAM_BAG_END;
  if (got != 4) return bag_fail(LOAM_E_INVAL, "bag: truncated record header length");
  const uint32_t hl = rd_u32(len4);
  hdr.resize(hl);
  if (hl && std::fread(hdr.data(), 1, hl, b->f) != hl) return bag_fail(LOAM_E_INVAL, "bag: truncated record header");
  if (std::fread(len4, 1, 4, b->f) != 4) return bag_fail(LOAM_E_INVAL, "bag: truncated record data length");
  const uint32_t dl = rd_u32(len4);
  data.resize(dl);
  if (dl && std::fread(data.data(), 1, dl, b->f) != dl) return bag_fail(LOAM_E_INVAL, "bag: truncated record data");
  return LOAM_OK;
}

int decompress(const std::string& comp, const std::vector<uint8_t>& in, uint32_t size, std::vector<uint8_t>& out) {
  out.resize(size);
  if (comp == "none") {
    if (in.size() != size) return bag_fail(LOAM_E_INVAL, "bag: uncompressed chunk size mismatch");
    if (size) std::memcpy(out.data(), in.data(), size);
    return LOAM_OK;
  }
  if (comp == "bz2") {
    if (!g_codecs.load_bz2()) return bag_fail(LOAM_E_INVAL, "bag: bz2 chunk but libbz2.so.1 is not available");
    unsigned n = size;
    const int rc = g_codecs.bz_decompress((char*)out.data(), &n, (char*)in.data(), (unsigned)in.size(), 0, 0);
    if (rc != 0 || n != size) return bag_fail(LOAM_E_INVAL, "bag: bz2 chunk does not decompress");
    return LOAM_OK;
  }
  if (comp == "lz4") {
    if (!g_codecs.load_lz4()) return bag_fail(LOAM_E_INVAL, "bag: lz4 chunk but liblz4.so.1 is not available");
    void* ctx = nullptr;
    if (g_codecs.lz4f_iserror(g_codecs.lz4f_create(&ctx, 100 /* LZ4F_VERSION */)))
      return bag_fail(LOAM_E_INVAL, "bag: lz4 context");
    size_t src_pos = 0, dst_pos = 0;
    bool ok = true;
    while (src_pos < in.size() && dst_pos <= size) {
      size_t dn = size - dst_pos, sn = in.size() - src_pos;
      const size_t r = g_codecs.lz4f_decompress(ctx, out.data() + dst_pos, &dn, in.data() + src_pos, &sn, nullptr);
      if (g_codecs.lz4f_iserror(r)) { ok = false; break; }
      src_pos += sn;
      dst_pos += dn;
      if (r == 0) break;  // frame complete
      if (sn == 0 && dn == 0) { ok = false; break; }
    }
    g_codecs.lz4f_free(ctx);
    if (!ok || dst_pos != size) return bag_fail(LOAM_E_INVAL, "bag: lz4 chunk does not decompress");
    return LOAM_OK;
  }
  return bag_fail(LOAM_E_INVAL, "bag: unknown chunk compression '" + comp + "'");
}

int add_connection(loam_bag* b, const Fields& h, const uint8_t* data, uint32_t n) {
  uint32_t conn;
  if (!h.u32("conn", conn)) return bag_fail(LOAM_E_INVAL, "bag: connection record without conn");
  Fields c;
  if (!c.parse(data, n)) return bag_fail(LOAM_E_INVAL, "bag: malformed connection header");
  std::string topic = h.str("topic");
  if (topic.empty()) topic = c.str("topic");
  b->conns[conn] = {topic, c.str("type")};
  return LOAM_OK;
}

}  // namespace

extern "C" {

int loam_bag_open(loam_bag** out, const char* path) {
  if (!out || !path) return bag_fail(LOAM_E_INVAL, "null argument");
  *out = nullptr;
  FILE* f = std::fopen(path, "rb");
  if (!f) return bag_fail(LOAM_E_INVAL, std::string("bag: cannot open ") + path);
  char magic[13];
  if (std::fread(magic, 1, 13, f) != 13 || std::memcmp(magic, "#ROSBAG V2.0\n", 13) != 0) {
    std::fclose(f);
    return bag_fail(LOAM_E_INVAL, "bag: not a rosbag v2.0 file");
  }
  loam_bag* b = new loam_bag();
  b->f = f;
  *out = b;
  return LOAM_OK;
}

void loam_bag_close(loam_bag* b) {
  if (!b) return;
  if (b->f) std::fclose(b->f);
  delete b;
}

int loam_bag_next(loam_bag* b, loam_bag_msg* m) {
  if (!b || !m) return bag_fail(LOAM_E_INVAL, "null argument");
  for (;;) {
    const uint8_t *hp, *dp;
    uint32_t hl, dl;
    bool in_chunk = false;
    if (b->chunk_pos < b->chunk.size()) {  // next record inside the current chunk
      const size_t n = b->chunk.size(), p = b->chunk_pos;
      if (n - p < 4) return bag_fail(LOAM_E_INVAL, "bag: truncated chunk record");
      hl = rd_u32(&b->chunk[p]);
      if (hl > n - p - 4 || n - p - 4 - hl < 4) return bag_fail(LOAM_E_INVAL, "bag: truncated chunk record");
      hp = &b->chunk[p + 4];
      dl = rd_u32(&b->chunk[p + 4 + hl]);
      if (dl > n - p - 8 - hl) return bag_fail(LOAM_E_INVAL, "bag: truncated chunk record data");
      dp = &b->chunk[p + 8 + hl];
      b->chunk_pos = p + 8 + hl + dl;
      in_chunk = true;
    } else {
      const int rc = read_record(b, b->rec_hdr, b->rec_data);
      if (rc != LOAM_OK) return rc;
      hp = b->rec_hdr.data();
      hl = (uint32_t)b->rec_hdr.size();
      dp = b->rec_data.data();
      dl = (uint32_t)b->rec_data.size();
    }
    Fields h;
    if (!h.parse(hp, hl)) return bag_fail(LOAM_E_INVAL, "bag: malformed record header");
    uint8_t op;
    if (!h.u8("op", op)) return bag_fail(LOAM_E_INVAL, "bag: record without op");
    if (op == 0x05 && !in_chunk) {  // chunk
      uint32_t size;
      if (!h.u32("size", size)) return bag_fail(LOAM_E_INVAL, "bag: chunk without size");
      std::vector<uint8_t> out;
      const int rc = decompress(h.str("compression"), b->rec_data, size, out);
      if (rc != LOAM_OK) return rc;
      b->chunk.swap(out);
      b->chunk_pos = 0;
      continue;
    }
    if (op == 0x07) {  // connection
      const int rc = add_connection(b, h, dp, dl);
      if (rc != LOAM_OK) return rc;
      continue;
    }
    if (op != 0x02) continue;  // bag header, index data, chunk info
    uint32_t conn;
    if (!h.u32("conn", conn)) return bag_fail(LOAM_E_INVAL, "bag: message without conn");
    auto it = b->conns.find(conn);
    if (it == b->conns.end()) return bag_fail(LOAM_E_INVAL, "bag: message on an unknown connection");
    auto tf = h.f.find("time");
    if (tf == h.f.end() || tf->second.second < 8) return bag_fail(LOAM_E_INVAL, "bag: message without time");
    const uint32_t sec = rd_u32(tf->second.first), nsec = rd_u32(tf->second.first + 4);
    b->msg.assign(dp, dp + dl);
    m->topic = it->second.first.c_str();
    m->type = it->second.second.c_str();
    m->stamp = (double)sec + 1e-9 * (double)nsec;
    m->data = b->msg.data();
    m->size = dl;
    return LOAM_OK;
  }
}

// ---- ROS1 serialization (little endian): u32 / f64 fields, strings and arrays as u32 length + bytes
namespace {
struct Rd {
  const uint8_t* p;
  uint32_t n, i = 0;
  bool ok = true;
  bool need(uint32_t k) {
    if (!ok || k > n - i) ok = false;
    return ok;
  }
  uint32_t u32() {
    if (!need(4)) return 0;
    const uint32_t v = rd_u32(p + i);
    i += 4;
    return v;
  }
  uint8_t u8() {
    if (!need(1)) return 0;
    return p[i++];
  }
  double f64() {
    if (!need(8)) return 0.0;
    double v;
    std::memcpy(&v, p + i, 8);
    i += 8;
    return v;
  }
  std::string str() {
    const uint32_t k = u32();
    if (!need(k)) return std::string();
    std::string s((const char*)p + i, k);
    i += k;
    return s;
  }
  double stamp() {  // std_msgs/Header: seq, stamp (sec, nsec), frame_id
    (void)u32();
    const uint32_t sec = u32(), nsec = u32();
    (void)str();
    return (double)sec + 1e-9 * (double)nsec;
  }
};
}  // namespace

int loam_pc2_parse(const uint8_t* msg, uint32_t size, loam_pc2* out) {
  if (!msg || !out) return bag_fail(LOAM_E_INVAL, "null argument");
  Rd r{msg, size};
  loam_pc2 pc;
  std::memset(&pc, 0, sizeof(pc));
  pc.off_x = pc.off_y = pc.off_z = pc.off_intensity = pc.off_ring = -1;
  pc.stamp = r.stamp();
  pc.height = r.u32();
  pc.width = r.u32();
  const uint32_t nf = r.u32();
  bool xyz_f32 = true;
  for (uint32_t k = 0; k < nf && r.ok; ++k) {
    const std::string name = r.str();
    const uint32_t off = r.u32();
    const uint8_t dtype = r.u8();  // sensor_msgs/PointField: 7 = FLOAT32
    (void)r.u32();                 // count
    if (name == "x" || name == "y" || name == "z") {
      if (dtype != 7) xyz_f32 = false;
      (name == "x" ? pc.off_x : name == "y" ? pc.off_y : pc.off_z) = (int32_t)off;
    } else if (name == "intensity") {
      pc.off_intensity = (int32_t)off;
    } else if (name == "ring") {
      pc.off_ring = (int32_t)off;
    }
  }
  pc.is_bigendian = r.u8();
  pc.point_step = r.u32();
  pc.row_step = r.u32();
  const uint32_t nd = r.u32();
  if (r.need(nd)) {
    pc.data = msg + r.i;
    pc.data_size = nd;
    r.i += nd;
  }
  pc.is_dense = r.u8();
  if (!r.ok) return bag_fail(LOAM_E_INVAL, "PointCloud2: truncated message");
  if (pc.off_x < 0 || pc.off_y < 0 || pc.off_z < 0 || !xyz_f32)
    return bag_fail(LOAM_E_INVAL, "PointCloud2: x / y / z FLOAT32 fields required");
  if (pc.is_bigendian) return bag_fail(LOAM_E_INVAL, "PointCloud2: big-endian clouds are not supported");
  const uint64_t npts = (uint64_t)pc.width * pc.height;
  if (pc.point_step < 12 || (uint64_t)pc.off_x + 4 > pc.point_step || (uint64_t)pc.off_y + 4 > pc.point_step ||
      (uint64_t)pc.off_z + 4 > pc.point_step || npts * pc.point_step > pc.data_size)
    return bag_fail(LOAM_E_INVAL, "PointCloud2: point layout does not fit the data");
  *out = pc;
  return LOAM_OK;
}

int loam_pc2_cloud(const loam_pc2* pc, loam_point* scratch, uint32_t scratch_cap, loam_cloud_in* out) {
  if (!pc || !out) return bag_fail(LOAM_E_INVAL, "null argument");
  const uint64_t n = (uint64_t)pc->width * pc->height;
  if (n > 0xffffffffull) return bag_fail(LOAM_E_INVAL, "PointCloud2: too many points");
  // the C-ABI's record layout already: hand the message over (at any alignment: the data follows
  // the message's variable-length header; the engine reads the records with unaligned copies)
  if (pc->off_x == 0 && pc->off_y == 4 && pc->off_z == 8 && pc->point_step >= 12 && (pc->point_step & 3) == 0) {
    out->data = pc->data;
    out->count = (uint32_t)n;
    out->stride_bytes = pc->point_step;
    return LOAM_OK;
  }
  if (!scratch || scratch_cap < n) {
    out->count = (uint32_t)n;
    return bag_fail(LOAM_E_CAPACITY, "PointCloud2: x / y / z not at offsets 0 / 4 / 8; scratch too small to pack");
  }
  for (uint64_t i = 0; i < n; ++i) {  // like pcl::fromROSMsg: fields copied by name
    const uint8_t* rec = pc->data + i * pc->point_step;
    std::memcpy(&scratch[i].x, rec + pc->off_x, 4);
    std::memcpy(&scratch[i].y, rec + pc->off_y, 4);
    std::memcpy(&scratch[i].z, rec + pc->off_z, 4);
    scratch[i].intensity = 0.0f;
    if (pc->off_intensity >= 0 && (uint32_t)pc->off_intensity + 4 <= pc->point_step)
      std::memcpy(&scratch[i].intensity, rec + pc->off_intensity, 4);
  }
  out->data = scratch;
  out->count = (uint32_t)n;
  out->stride_bytes = sizeof(loam_point);
  return LOAM_OK;
}

int loam_imu_parse(const uint8_t* msg, uint32_t size, double* stamp, double quat_xyzw[4], double lin_acc[3]) {
  if (!msg || !stamp || !quat_xyzw || !lin_acc) return bag_fail(LOAM_E_INVAL, "null argument");
  Rd r{msg, size};
  const double t = r.stamp();
  double q[4], a[3];
  for (int k = 0; k < 4; ++k) q[k] = r.f64();       // orientation x, y, z, w
  for (int k = 0; k < 9; ++k) (void)r.f64();        // orientation_covariance
  for (int k = 0; k < 3; ++k) (void)r.f64();        // angular_velocity
  for (int k = 0; k < 9; ++k) (void)r.f64();        // angular_velocity_covariance
  for (int k = 0; k < 3; ++k) a[k] = r.f64();       // linear_acceleration
  for (int k = 0; k < 9; ++k) (void)r.f64();        // linear_acceleration_covariance
  if (!r.ok) return bag_fail(LOAM_E_INVAL, "Imu: truncated message");
  *stamp = t;
  for (int k = 0; k < 4; ++k) quat_xyzw[k] = q[k];
  for (int k = 0; k < 3; ++k) lin_acc[k] = a[k];
  return LOAM_OK;
}

}  // extern "C"
