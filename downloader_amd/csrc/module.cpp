// pybind11 bindings for the stager host-native module `_native`.
// Every entry point that touches bytes releases the GIL so asyncio worker threads (and
// several jobs in one worker process) run hashing and transfers truly in parallel.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <cstdlib>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>

#include "native.h"

namespace py = pybind11;
using namespace stager;

namespace {

struct BufView {
  const uint8_t* p;
  size_t n;
  py::buffer_info info;  // keeps the exporter alive/locked
};

BufView view(const py::buffer& b) {
  py::buffer_info info = b.request();
  if (info.ndim > 1 && info.strides.back() != info.itemsize)
    throw std::invalid_argument("buffer must be C-contiguous");
  size_t n = (size_t)info.size * (size_t)info.itemsize;
  return BufView{(const uint8_t*)info.ptr, n, std::move(info)};
}

py::dict head_to_dict(const ResponseHead& h) {
  py::dict d;
  d["status"] = h.status;
  d["reason"] = h.reason;
  py::list hs;
  for (auto& kv : h.headers) hs.append(py::make_tuple(kv.first, kv.second));
  d["headers"] = hs;
  d["content_length"] = h.content_length;
  d["chunked"] = h.chunked;
  d["keep_alive"] = h.keep_alive;
  return d;
}

}  // namespace

// The relay failed after queueing its part to the GPU hasher: nobody asks for the digests.
// Returns once the part's buffer is back in the pool (its DMA is over).
void forget_ticket(uint64_t id) {
  if (id) gpu_part_forget(id);
}

// STAGER_FAULT_BAD_CRC=<pattern>[:count] (fault injection for the integrity tests): the
// CRC32C trailer of the next `count` (default 1) relayed PUTs whose request head matches
// `pattern` (substrings joined by '*', found in that order) goes out with one bit flipped, as a
// corrupting hop between the worker's CRC and the socket would send it. The S3 side must
// refuse it (400 BadDigest).
static bool head_matches(const std::string& head, const std::string& pat) {
  size_t at = 0, i = 0;
  while (i <= pat.size()) {
    size_t star = pat.find('*', i);
    if (star == std::string::npos) star = pat.size();
    std::string piece = pat.substr(i, star - i);
    if (!piece.empty()) {
      size_t f = head.find(piece, at);
      if (f == std::string::npos) return false;
      at = f + piece.size();
    }
    i = star + 1;
  }
  return true;
}

static bool fault_bad_crc(const std::string& put_head) {
  static std::string pat;
  static std::atomic<int64_t> left{[] {
    const char* e = getenv("STAGER_FAULT_BAD_CRC");
    if (!e || !*e) return (int64_t)0;
    std::string v(e);
    size_t c = v.rfind(':');
    int64_t n = 1;
    if (c != std::string::npos && c + 1 < v.size() &&
        v.find_first_not_of("0123456789", c + 1) == std::string::npos) {
      n = atoll(v.c_str() + c + 1);
      v.resize(c);
    }
    pat = v;
    return n;
  }()};
  if (left.load(std::memory_order_relaxed) <= 0 || !head_matches(put_head, pat)) return false;
  return left.fetch_sub(1) > 0;
}

struct PieceSplit {
  int64_t skip, full_len, piece_len;
};

// GET on `src`, then (only on 200/206 with exactly `length` bytes) the PUT head on `dst`
// followed by the body: spliced socket->pipe->socket, or - with `split` - through a hashed
// user-space chunk (HttpConn::relay_body_hashed).
// `crc`: the PUT is aws-chunked (the head carries the encoded Content-Length): one data chunk,
// then a zero chunk whose trailer is the CRC32C of the bytes moved (x-amz-checksum-crc32c).
py::dict relay(HttpConn& src, const py::bytes& get_head, HttpConn& dst, const py::bytes& put_head,
               int64_t length, Progress* prog, int64_t max_body, const PieceSplit* split,
               bool crc, bool gpu = false) {
  std::string gh = get_head, ph = put_head;
  ResponseHead g, p;
  std::string gerr, pbody, digests, head, tail, crc_b64;
  int64_t moved = 0;
  uint64_t ticket = 0;
  {
    py::gil_scoped_release rel;
    try {
      src.send_request(gh, nullptr, 0);
      g = src.read_head();
      bool ok = (g.status == 200 || g.status == 206) && !g.chunked && g.content_length == length;
      if (!ok) {
        // an error page is read for the message; a big unwanted body (a whole 200 where a 206
        // slice was asked - If-Range on a changed source) is not: the connection is dropped
        if (!g.chunked && g.content_length >= 0 && g.content_length <= (1 << 20))
          gerr = src.read_body(g, 1 << 20);
        else
          src.mark_unusable();
      } else {
        int cork = 1;
        setsockopt(dst.fd(), IPPROTO_TCP, TCP_CORK, &cork, sizeof(cork));
        dst.send_raw(ph);
        uint32_t c = 0;
        if (crc && length > 0) {
          char hx[32];
          snprintf(hx, sizeof hx, "%llx\r\n", (unsigned long long)length);
          dst.send_raw(hx);
        }
        moved = split ? src.relay_body_hashed(dst, length, split->skip, split->full_len,
                                              split->piece_len, prog, &digests, &head, &tail,
                                              crc ? &c : nullptr, gpu ? &ticket : nullptr)
                      : src.relay_body_to(dst, length, prog, crc ? &c : nullptr);
        if (crc) {
          if (fault_bad_crc(ph)) c ^= 1u;
          crc_b64 = crc32c_base64(c);
          dst.send_raw(std::string(length > 0 ? "\r\n" : "") + "0\r\nx-amz-checksum-crc32c:" +
                       crc_b64 + "\r\n\r\n");
        }
        cork = 0;
        setsockopt(dst.fd(), IPPROTO_TCP, TCP_CORK, &cork, sizeof(cork));
        p = dst.read_head();
        pbody = dst.read_body(p, max_body);
      }
    } catch (...) {
      forget_ticket(ticket);
      throw;
    }
    // a refused PUT is retried from the GET: its queued digests are never asked for
    if (ticket && !(p.status >= 200 && p.status < 300)) {
      forget_ticket(ticket);
      ticket = 0;
    }
  }
  py::dict d;
  d["get"] = head_to_dict(g);
  d["get_body"] = py::bytes(gerr);
  d["put"] = p.status ? (py::object)head_to_dict(p) : py::none();
  d["put_body"] = py::bytes(pbody);
  d["moved"] = moved;
  d["crc32c"] = crc_b64;
  if (split) {
    d["gpu_ticket"] = ticket;      // != 0: a part id; digests via gpu_part_poll / gpu_part_wait
    d["digests"] = py::bytes(digests);
    d["head"] = py::bytes(head);
    d["tail"] = py::bytes(tail);
  }
  return d;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "stager host-native byte paths: hashing (OpenSSL EVP, threaded) and zero-copy HTTP";

  m.def("digest_size", &digest_size);
  m.def("crc32c_impl", []() { return std::string(crc32c_impl()); },
        "the CRC32C implementation this CPU runs (avx512-vpclmulqdq / sse4.2-3way)");
  m.def("sha1_mb_supported", &sha1_mb_supported,
        "True when the host runs the AVX-512 16-lane multi-buffer SHA-1 (csrc/sha1_mb.cpp)");
  m.def("effective_cpus", &effective_cpus,
        "CPUs usable by this process: affinity mask capped by the cgroup v2 cpu.max quota");
  m.def(
      "set_gpu_part_hasher",
      [](const py::object& capsule, int min_pieces) {
        if (capsule.is_none()) {
          set_gpu_part_hasher(nullptr, min_pieces);
          return;
        }
        void* p = PyCapsule_GetPointer(capsule.ptr(), "downloader_amd.gpu_part_api");
        if (!p) throw py::error_already_set();
        set_gpu_part_hasher(p, min_pieces);
      },
      py::arg("api"), py::arg("min_pieces") = 8,
      "Route the hashed relay's parts (>= min_pieces whole pieces) to the GPU hasher whose C "
      "ABI capsule is `api` (_gpuhash.PartHasher.api()); None: host multi-buffer SHA-1");
  m.def(
      "gpu_part_wait",
      [](uint64_t id) {
        std::string d;
        {
          py::gil_scoped_release rel;
          d = gpu_part_wait(id);
        }
        return py::bytes(d);
      },
      py::arg("id"), "Block until part `id` (the relay's gpu_ticket) is hashed: its digests");
  m.def(
      "gpu_part_forget",
      [](uint64_t id) {
        py::gil_scoped_release rel;
        gpu_part_forget(id);
      },
      py::arg("id"),
      "Nobody will ask for part `id`: returns once its buffer is back in the pool; the result "
      "is dropped when it arrives");
  m.def("gpu_part_eventfd", &gpu_part_eventfd,
        "eventfd that turns readable when gpu_part_poll has news");
  m.def(
      "gpu_part_poll",
      []() {
        std::vector<GpuPartEvent> ev;
        {
          py::gil_scoped_release rel;
          ev = gpu_part_poll();
        }
        py::list out;
        for (auto& e : ev)
          out.append(py::make_tuple(e.id, e.kind, py::bytes(e.data)));
        return out;
      },
      "Drain completions: [(id, kind, data)] with kind 1 = copied (the part's buffer is back in "
      "the pool), 2 = done (data = 20 B digests per piece), 3 = failed (data = error message)");
  py::class_<CpuPartHasher>(m, "CpuPartHasher")
      .def(py::init<double, int, int>(), py::arg("delay_s") = 0.005,
           py::arg("fail_copy_every") = 0, py::arg("fail_done_every") = 0,
           "gpu_part_api.h on a host thread (tests of the asynchronous relay-hashing path); "
           "fail_*_every: every Nth job's copy / hash fails")
      .def("api", [](CpuPartHasher& h) {
        return py::capsule((void*)h.api(), "downloader_amd.gpu_part_api");
      })
      .def_property_readonly("registered", &CpuPartHasher::registered);
  m.def("gpu_part_stats", []() {
    GpuPartStats s = gpu_part_stats();
    py::dict d;
    d["submitted"] = s.submitted;
    d["host_fallbacks"] = s.host_fallbacks;
    d["refused"] = s.refused;
    d["pending"] = s.pending;
    return d;
  });
  m.def("relay_pool_trim", &relay_pool_trim, py::arg("keep_bytes") = 0,
        "Unmap idle hashed-relay part buffers beyond keep_bytes; returns the bytes freed");
  m.def("relay_pool_set_budget", &relay_pool_set_budget, py::arg("bytes"),
        "Bound leased + idle part buffers (0 = no bound): idle ones are unmapped to make room");
  m.def("relay_pool_reset_peak", &relay_pool_reset_peak,
        "Restart the pool's high-water mark (peak_bytes) and its over_budget count");
  m.def("relay_pool_set_max_idle", &relay_pool_set_max_idle, py::arg("n"),
        "Keep at most n idle part buffers (the rest are unmapped on release)");
  py::class_<SwarmWire>(m, "SwarmWire",
                        "Native peer-wire receive path of one torrent session (peerwire.cpp)")
      .def(py::init<int, int>(), py::arg("verify_threads") = 2, py::arg("io_threads") = 4)
      .def("set_storage",
           [](SwarmWire& w, int64_t piece_length, int64_t total, const py::bytes& hashes,
              const std::vector<std::pair<int, int64_t>>& files) {
             w.set_storage(piece_length, total, std::string(hashes), files);
           },
           py::arg("piece_length"), py::arg("total"), py::arg("hashes"), py::arg("files"))
      .def("begin_piece", &SwarmWire::begin_piece, py::arg("idx"))
      .def("drop_piece", &SwarmWire::drop_piece, py::arg("idx"))
      .def("set_pipeline", &SwarmWire::set_pipeline, py::arg("depth"))
      .def("set_conn_pipeline", &SwarmWire::set_conn_pipeline, py::arg("conn_id"),
           py::arg("depth"), "requests in flight on one connection (its bandwidth-delay product)")
      .def("assign", &SwarmWire::assign, py::arg("conn_id"), py::arg("idx"),
           "Own piece idx on the connection: the wire requests its blocks (returns the "
           "connection's blocks still to request)")
      .def("todo", &SwarmWire::todo, py::arg("conn_id"))
      .def("release",
           [](SwarmWire& w, uint64_t id) {
             py::list out;
             for (auto& r : w.release(id)) out.append(py::make_tuple(r.first, py::bytes(r.second)));
             return out;
           },
           py::arg("conn_id"),
           "[(idx, states)] of the pieces the connection owned, now ordinary (2 received, "
           "1 requested and unanswered, 0 neither)")
      .def("release_piece",
           [](SwarmWire& w, uint32_t idx) -> py::object {
             uint64_t owner = 0;
             std::string st;
             if (!w.release_piece(idx, &owner, &st)) return py::none();
             return py::make_tuple(owner, py::bytes(st));
           },
           py::arg("idx"), "(owner, states) of an owned piece made ordinary, or None")
      .def("rx_idle", &SwarmWire::rx_idle, py::arg("conn_id"))
      .def("take_block",
           [](SwarmWire& w, uint32_t idx, uint32_t begin, const py::buffer& b) {
             py::buffer_info i = b.request();
             return w.take_block(idx, begin, (const uint8_t*)i.ptr,
                                 (uint32_t)(i.size * i.itemsize));
           },
           py::arg("idx"), py::arg("begin"), py::arg("data"),
           "A block received on a Python-framed connection: 0 not taken, 1 taken, 2 taken "
           "and the piece complete")
      .def("set_have",
           [](SwarmWire& w, const py::bytes& bits) { w.set_have(std::string(bits)); },
           py::arg("bits"))
      .def("set_have_piece", &SwarmWire::set_have_piece, py::arg("idx"))
      .def("set_serving", &SwarmWire::set_serving, py::arg("conn_id"), py::arg("on"))
      .def("set_backlog_cap", &SwarmWire::set_backlog_cap, py::arg("bytes"))
      .def("backlogged", &SwarmWire::backlogged,
           "True while complete, unreported pieces hold the cap or more (start no new piece)")
      .def("set_host_tail", &SwarmWire::set_host_tail, py::arg("on"),
           "GPU mode: hash the pieces completing from now on on the host (the download's end)")
      .def("rx_total", &SwarmWire::rx_total, "bytes received on every connection so far")
      .def("gpu_latency", &SwarmWire::gpu_latency,
           "GPU mode: submission -> digest time of the device's pieces (EWMA, s; 0 = none yet)")
      .def("set_gpu", &SwarmWire::set_gpu, py::arg("on"), py::arg("max_inflight") = 64,
           "Verify complete pieces on the installed GPU part hasher (set_gpu_part_hasher), at "
           "most max_inflight at once (the rest on the host)")
      .def("attach",
           [](SwarmWire& w, int fd, uint64_t id, const py::bytes& prefix) {
             w.attach(fd, id, std::string(prefix));
           },
           py::arg("fd"), py::arg("conn_id"), py::arg("prefix") = py::bytes(),
           "Hand a connected socket over (the fd is owned from here on, closed by detach)")
      .def("send",
           [](SwarmWire& w, uint64_t id, const py::bytes& data) {
             std::string s(data);
             return w.send(id, std::move(s));
           },
           py::arg("conn_id"), py::arg("data"))
      .def("sendv",
           [](SwarmWire& w, uint64_t id, const py::list& parts) {
             // one copy of the parts (bytes, memoryviews of cached pieces) into the queue
             size_t n = 0;
             std::vector<py::buffer_info> infos;
             infos.reserve(parts.size());
             for (auto h : parts) {
               infos.push_back(py::reinterpret_borrow<py::buffer>(h).request());
               n += (size_t)infos.back().size * (size_t)infos.back().itemsize;
             }
             std::string s;
             s.reserve(n);
             for (auto& i : infos) s.append((const char*)i.ptr, (size_t)i.size * (size_t)i.itemsize);
             return w.send(id, std::move(s));
           },
           py::arg("conn_id"), py::arg("parts"),
           "Queue the concatenation of `parts` (buffers) for sending; the queued bytes after it")
      .def("pending_out", &SwarmWire::pending_out, py::arg("conn_id"))
      .def("conn_rx", &SwarmWire::conn_rx, py::arg("conn_id"),
           "bytes the connection received so far (per-peer rates)")
      .def("detach", &SwarmWire::detach, py::arg("conn_id"),
           py::call_guard<py::gil_scoped_release>())
      .def("eventfd", &SwarmWire::eventfd)
      .def("poll",
           [](SwarmWire& w) {
             std::vector<WireEvent> ev = w.poll();
             py::list out;
             for (auto& e : ev) out.append(py::make_tuple(e.conn, e.kind, py::bytes(e.data)));
             return out;
           },
           "[(conn_id, kind, data)]: 1 message, 2 blocks, 3 closed, 4 piece (conn 0), "
           "5 the connection's request queue runs low")
      .def("stats",
           [](SwarmWire& w) {
             SwarmWireStats s = w.stats();
             py::dict d;
             d["begun"] = s.begun;
             d["blocks"] = s.blocks;
             d["block_bytes"] = s.block_bytes;
             d["blocks_ignored"] = s.blocks_ignored;
             d["verified"] = s.verified;
             d["hash_fails"] = s.hash_fails;
             d["rx_bytes"] = s.rx_bytes;
             d["recvs"] = s.recvs;
             d["active_pieces"] = s.active_pieces;
             d["verify_batches"] = s.verify_batches;
             d["sha_s"] = s.sha_ns / 1e9;
             d["write_s"] = s.write_ns / 1e9;
             d["served_bytes"] = s.served_bytes;
             d["io_threads"] = s.io_threads;
             d["serve_floods"] = s.serve_floods;
             d["serve_cancels"] = s.serve_cancels;
             d["assigned"] = s.assigned;            // owned pieces (SwarmWire.assign)
             d["requests"] = s.requests;            // REQUESTs the wire sent by itself
             d["gpu_pieces"] = s.gpu_pieces;
             d["gpu_refused"] = s.gpu_refused;
             d["gpu_errors"] = s.gpu_errors;
             d["gpu_overflow"] = s.gpu_overflow;    // hashed on the host: device full
             d["gpu_latency_ms_mean"] =
                 s.gpu_pieces ? s.gpu_latency_ns_sum / 1e6 / (double)s.gpu_pieces : 0.0;
             d["gpu_latency_ms_max"] = s.gpu_latency_ns_max / 1e6;
             d["backlog_bytes"] = s.backlog_bytes;
             d["pool_in_use"] = s.pool_in_use;      // process-wide piece buffers
             d["pool_idle"] = s.pool_idle;
             d["pool_idle_bytes"] = s.pool_idle_bytes;
             d["pool_allocs"] = s.pool_allocs;      // (process lifetime)
             d["pool_frees"] = s.pool_frees;
             d["pool_locks"] = s.pool_locks;
             return d;
           })
      .def("close", &SwarmWire::close, py::call_guard<py::gil_scoped_release>());
  m.def("swarm_piece_pool_limit", &swarm_piece_pool_limit, py::arg("bytes"),
        "Keep at most `bytes` of idle swarm piece buffers (process-wide; the rest are freed)");
  m.def("relay_counters", []() {
    RelayCounters c = relay_counters();
    py::dict d;
    const char* modes[4] = {"splice", "dup", "copy", "hashed"};
    for (int i = 0; i < 4; ++i) {
      d[(std::string(modes[i]) + "_relays").c_str()] = c.relays[i];
      d[(std::string(modes[i]) + "_bytes").c_str()] = c.bytes[i];
      d[(std::string(modes[i]) + "_cpu_ns").c_str()] = c.cpu_ns[i];
    }
    d["splice_in_calls"] = c.splice_in_calls;
    d["splice_out_calls"] = c.splice_out_calls;
    d["dup_calls"] = c.dup_calls;
    d["dup_copied_bytes"] = c.dup_bytes;
    d["crc_ns"] = c.crc_ns;
    d["crc_bytes"] = c.crc_bytes;
    d["sha1_ns"] = c.sha1_ns;
    d["nt_staged_bytes"] = c.nt_bytes;
    return d;
  }, "Per-phase relay counters since start (relay_body_to): relays / bytes / relaying-thread "
     "CPU per mode (splice, dup = peek|tee copy + CRC, copy), syscalls, copy and CRC time");
  m.def("pipe_stats", []() {
    PipeStats s = pipe_stats();
    py::dict d;
    d["created"] = s.created;
    d["short"] = s.short_pipes;
    d["in_use"] = s.in_use;
    d["in_use_bytes"] = s.in_use_bytes;
    d["idle"] = s.idle;
    d["idle_bytes"] = s.idle_bytes;
    return d;
  }, "splice pipes: created, created below the asked capacity (the user's pipe page budget, "
     "fs.pipe-user-pages-soft, is spent), leased / idle and their capacity");
  m.def("set_pipes_refused", &set_pipes_refused,
        "tests: refuse every splice pipe as if the user's pipe budget were spent");
  m.def("set_relay_dup", &set_relay_dup, py::arg("mode"),
        "relays that need the bytes (CRC, piece hashing): 'peek' (recv(MSG_PEEK) + splice, one "
        "pipe) or 'tee' (tee() into a second pipe)");
  m.def("relay_dup_mode", &relay_dup_mode);
  m.def("set_pipe_sizes", &set_pipe_sizes, py::arg("main"), py::arg("tee") = 0,
        "capacity asked for new splice pipes and tee() duplicate pipes (0 = keep)");
  m.def("relay_pool_stats", []() {
    RelayPoolStats s = relay_pool_stats();
    py::dict d;
    d["idle_buffers"] = s.idle_buffers;
    d["idle_bytes"] = s.idle_bytes;
    d["in_use"] = s.in_use;
    d["max_idle"] = s.max_idle;
    d["created"] = s.created;
    d["in_use_bytes"] = s.in_use_bytes;
    d["budget"] = s.budget;
    d["peak_bytes"] = s.peak_bytes;
    d["evicted"] = s.evicted;
    d["over_budget"] = s.over_budget;
    return d;
  });
  m.def(
      "digest",
      [](const std::string& algo, const py::buffer& data) {
        BufView v = view(data);
        std::string out;
        {
          py::gil_scoped_release rel;
          out = digest(algo, v.p, v.n);
        }
        return py::bytes(out);
      },
      py::arg("algo"), py::arg("data"));
  m.def(
      "crc32c",
      [](const py::buffer& data, uint32_t crc) {
        BufView v = view(data);
        if (v.n < 65536) return crc32c(v.p, v.n, crc);
        py::gil_scoped_release rel;
        return crc32c(v.p, v.n, crc);
      },
      py::arg("data"), py::arg("crc") = 0,
      "CRC32C (Castagnoli) of data, continuing from `crc` (SSE4.2, three interleaved chains).");
  m.def(
      "crc32c_fd",
      [](int fd, int64_t off, int64_t len) {
        py::gil_scoped_release rel;
        return crc32c_fd(fd, off, len);
      },
      py::arg("fd"), py::arg("offset"), py::arg("length"), "CRC32C of a file range.");
  m.def("crc32c_base64", &crc32c_base64, py::arg("crc"),
        "x-amz-checksum-crc32c value: base64 of the big-endian CRC.");
  m.def(
      "hash_pieces",
      [](const std::string& algo, const py::buffer& data, size_t piece_len, int threads) {
        BufView v = view(data);
        std::string out;
        {
          py::gil_scoped_release rel;
          out = hash_pieces(algo, v.p, v.n, piece_len, threads);
        }
        return py::bytes(out);
      },
      py::arg("algo"), py::arg("data"), py::arg("piece_len"), py::arg("threads") = 0,
      "Concatenated per-piece digests of a contiguous buffer.");
  m.def(
      "verify_pieces",
      [](const std::vector<std::pair<std::string, int64_t>>& files, int64_t piece_len,
         const py::bytes& hashes, const std::vector<int64_t>& which, int threads) {
        std::string hs = hashes;
        std::vector<uint8_t> ok;
        {
          py::gil_scoped_release rel;
          ok = verify_pieces(files, piece_len, hs, which, threads);
        }
        return py::bytes((const char*)ok.data(), ok.size());
      },
      py::arg("files"), py::arg("piece_len"), py::arg("hashes"),
      py::arg("which") = std::vector<int64_t>{}, py::arg("threads") = 0,
      "SHA-1 verify torrent pieces stored across `files` [(path, length)]; returns one byte "
      "(0/1) per checked piece.");
  m.def(
      "hash_storage_pieces",
      [](const std::vector<std::pair<std::string, int64_t>>& files, int64_t piece_len,
         const std::string& algo, int threads) {
        std::string out;
        {
          py::gil_scoped_release rel;
          out = hash_storage_pieces(files, piece_len, algo, threads);
        }
        return py::bytes(out);
      },
      py::arg("files"), py::arg("piece_len"), py::arg("algo") = "sha1", py::arg("threads") = 0);
  m.def(
      "hash_file_ranges",
      [](const std::string& path, const std::vector<std::pair<int64_t, int64_t>>& ranges,
         const std::string& algo, int threads) {
        std::vector<std::string> out;
        {
          py::gil_scoped_release rel;
          out = hash_file_ranges(path, ranges, algo, threads);
        }
        py::list l;
        for (auto& s : out) l.append(py::bytes(s));
        return l;
      },
      py::arg("path"), py::arg("ranges"), py::arg("algo"), py::arg("threads") = 0);

  py::class_<Hasher>(m, "Hasher")
      .def(py::init<const std::string&>())
      .def("update",
           [](Hasher& h, const py::buffer& data) {
             BufView v = view(data);
             if (v.n >= 65536) {
               py::gil_scoped_release rel;
               h.update(v.p, v.n);
             } else {
               h.update(v.p, v.n);
             }
           })
      .def("update_fd",
           [](Hasher& h, int fd, int64_t off, int64_t len) {
             py::gil_scoped_release rel;
             h.update_fd(fd, off, len);
           })
      .def("digest", [](const Hasher& h) { return py::bytes(h.digest()); })
      .def("hexdigest",
           [](const Hasher& h) {
             std::string d = h.digest();
             static const char* hx = "0123456789abcdef";
             std::string s;
             for (unsigned char c : d) {
               s.push_back(hx[c >> 4]);
               s.push_back(hx[c & 15]);
             }
             return s;
           })
      .def("copy", [](const Hasher& h) { return h.copy(); })
      .def_property_readonly("name", &Hasher::algo);

  py::class_<Progress>(m, "Progress")
      .def(py::init<>())
      .def_property_readonly("bytes", [](const Progress& p) { return p.bytes.load(); })
      .def("cancel", [](Progress& p) { p.cancelled.store(true); })
      .def_property_readonly("cancelled", [](const Progress& p) { return p.cancelled.load(); });

  py::class_<TlsContext, std::shared_ptr<TlsContext>>(m, "TlsContext")
      .def(py::init<bool, const std::string&>(), py::arg("verify") = true,
           py::arg("ca_file") = "",
           "Client TLS settings shared by connections: verify peers against the system store "
           "plus ca_file (PEM), or not at all")
      .def_property_readonly("verify", &TlsContext::verify);

  py::class_<HttpConn>(m, "HttpConn", py::dynamic_attr())
      .def(py::init([](const std::string& host, int port, double cto, double iot,
                       std::shared_ptr<TlsContext> tls) {
             py::gil_scoped_release rel;
             return new HttpConn(host, port, cto, iot, std::move(tls));
           }),
           py::arg("host"), py::arg("port"), py::arg("connect_timeout") = 10.0,
           py::arg("io_timeout") = 300.0, py::arg("tls") = nullptr)
      .def(
          "request",
          [](HttpConn& c, const py::bytes& head, const py::object& body, bool expect_body,
             int64_t max_body) {
            std::string hs = head;
            std::string bs;
            if (!body.is_none()) bs = body.cast<std::string>();
            ResponseHead h;
            std::string rb;
            {
              py::gil_scoped_release rel;
              c.send_request(hs, (const uint8_t*)bs.data(), bs.size());
              h = c.read_head();
              if (expect_body) rb = c.read_body(h, max_body);
            }
            py::dict d = head_to_dict(h);
            d["body"] = py::bytes(rb);
            return d;
          },
          py::arg("head"), py::arg("body") = py::none(), py::arg("expect_body") = true,
          py::arg("max_body") = (int64_t)64 << 20,
          "Send a request with an in-memory body; return head + body.")
      .def(
          "request_fd",
          [](HttpConn& c, const py::bytes& head, int fd, int64_t off, int64_t len,
             Progress* prog, int64_t max_body) {
            std::string hs = head;
            ResponseHead h;
            std::string rb;
            {
              py::gil_scoped_release rel;
              c.send_request_fd(hs, fd, off, len, prog);
              h = c.read_head();
              rb = c.read_body(h, max_body);
            }
            py::dict d = head_to_dict(h);
            d["body"] = py::bytes(rb);
            return d;
          },
          py::arg("head"), py::arg("fd"), py::arg("offset"), py::arg("length"),
          py::arg("progress") = nullptr, py::arg("max_body") = (int64_t)64 << 20,
          "Send a request whose body is a file range (sendfile); return head + body.")
      .def(
          "get_to_fd",
          [](HttpConn& c, const py::bytes& head, int fd, int64_t off, int64_t max_bytes,
             Progress* prog, int64_t max_err_body) {
            std::string hs = head;
            ResponseHead h;
            int64_t n = 0;
            std::string err;
            {
              py::gil_scoped_release rel;
              c.send_request(hs, nullptr, 0);
              h = c.read_head();
              if (h.status >= 200 && h.status < 300 && !h.chunked && h.content_length > max_bytes)
                c.mark_unusable();   // more than asked (a 200 for a Range GET): not written
              else if (h.status >= 200 && h.status < 300)
                n = c.read_body_to_fd(h, fd, off, max_bytes, prog);
              else
                err = c.read_body(h, max_err_body);
            }
            py::dict d = head_to_dict(h);
            d["written"] = n;
            d["body"] = py::bytes(err);
            return d;
          },
          py::arg("head"), py::arg("fd"), py::arg("offset") = 0,
          py::arg("max_bytes") = (int64_t)1 << 50, py::arg("progress") = nullptr,
          py::arg("max_err_body") = (int64_t)1 << 20,
          "Send a body-less request; a 2xx body is spliced into `fd` at `offset`.")
      .def(
          "relay_to",
          [](HttpConn& src, const py::bytes& get_head, HttpConn& dst, const py::bytes& put_head,
             int64_t length, Progress* prog, int64_t max_body, bool crc) {
            return relay(src, get_head, dst, put_head, length, prog, max_body, nullptr, crc);
          },
          py::arg("get_head"), py::arg("dst"), py::arg("put_head"), py::arg("length"),
          py::arg("progress") = nullptr, py::arg("max_body") = (int64_t)1 << 20,
          py::arg("crc") = false,
          "GET on this connection and stream exactly `length` body bytes as the body of the "
          "PUT sent on `dst` (socket->pipe->socket splice). The GET must answer 200/206 with "
          "that Content-Length, otherwise nothing is sent on `dst`. crc=True: aws-chunked body "
          "with a trailing x-amz-checksum-crc32c (bytes through user space), returned as "
          "`crc32c` (base64).")
      .def(
          "relay_hashed_to",
          [](HttpConn& src, const py::bytes& get_head, HttpConn& dst, const py::bytes& put_head,
             int64_t length, int64_t skip, int64_t full_len, int64_t piece_len, Progress* prog,
             int64_t max_body, bool crc, bool gpu) {
            PieceSplit ps{skip, full_len, piece_len};
            return relay(src, get_head, dst, put_head, length, prog, max_body, &ps, crc, gpu);
          },
          py::arg("get_head"), py::arg("dst"), py::arg("put_head"), py::arg("length"),
          py::arg("skip"), py::arg("full_len"), py::arg("piece_len"),
          py::arg("progress") = nullptr, py::arg("max_body") = (int64_t)1 << 20,
          py::arg("crc") = false, py::arg("gpu") = false,
          "relay_to through a user-space chunk that is SHA-1'd on the way: body bytes "
          "[skip, skip+full_len) as consecutive `piece_len` pieces (last may be short). Adds "
          "`digests` (20 B per piece), `head` (bytes before skip) and `tail` (bytes after).")
      .def(
          "connect_tunnel",
          [](HttpConn& c, const std::string& target, const std::string& auth) {
            py::gil_scoped_release rel;
            c.connect_tunnel(target, auth);
          },
          py::arg("target"), py::arg("auth") = "",
          "CONNECT tunnel through the forward proxy this socket is connected to")
      .def(
          "start_tls",
          [](HttpConn& c, std::shared_ptr<TlsContext> tls, const std::string& name) {
            py::gil_scoped_release rel;
            c.start_tls(std::move(tls), name);
          },
          py::arg("tls"), py::arg("server_name"))
      .def("close", &HttpConn::close)
      .def("abort", &HttpConn::abort)
      .def_property_readonly("is_open", &HttpConn::is_open)
      .def_property_readonly("reusable", &HttpConn::reusable)
      .def_property_readonly("host", &HttpConn::host)
      .def_property_readonly("port", &HttpConn::port)
      .def_property_readonly("tls", &HttpConn::is_tls);
}
