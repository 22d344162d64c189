// TLS for the native HTTP transport: https:// origins and webseeds, S3 with `secure: true`,
// bucket:// sources (always TLS in the reference: lib/download.js:210 `useSSL: true`).
//
// Without this, every TLS byte went through aiohttp's ssl objects on the worker's event-loop
// thread: one core for all TLS streams of a process (~1.4 GB/s measured for one GET). Here a
// TLS connection is an HttpConn with an OpenSSL session on top of its blocking socket, driven
// by the transport's executor threads with the GIL released, so TLS streams scale with
// cores like the plain ones. What TLS takes away is the zero-copy path: bytes must pass
// through user space to be encrypted/decrypted (splice/sendfile -> read/pread + SSL_*);
// kernel TLS offload (TCP_ULP "tls") is not available on these hosts (tcp_available_ulp).
#include "native.h"

#include <arpa/inet.h>
#include <cerrno>
#include <cstring>
#include <openssl/err.h>
#include <openssl/ssl.h>
#include <openssl/x509v3.h>

#include <stdexcept>

namespace stager {

TlsContext::TlsContext(bool verify, const std::string& ca_file) : verify_(verify) {
  ctx_ = SSL_CTX_new(TLS_client_method());
  if (!ctx_) throw std::runtime_error("SSL_CTX_new failed");
  SSL_CTX_set_min_proto_version(ctx_, TLS1_2_VERSION);
  // HTTP framing (Content-Length / chunked) detects truncation; a peer that closes without
  // close_notify after a complete body is common and must not fail the transfer.
  SSL_CTX_set_options(ctx_, SSL_OP_IGNORE_UNEXPECTED_EOF | SSL_OP_NO_COMPRESSION);
  SSL_CTX_set_mode(ctx_, SSL_MODE_AUTO_RETRY);
  // AES-128-GCM first (OpenSSL's default order starts with AES-256): same security margin in
  // practice, fewer rounds per block; most servers (Go's crypto/tls, MinIO) prefer it anyway.
  SSL_CTX_set_ciphersuites(ctx_,
                           "TLS_AES_128_GCM_SHA256:TLS_AES_256_GCM_SHA384:TLS_CHACHA20_POLY1305_SHA256");
  // Read whole socket buffers into OpenSSL's record buffer: one recv per several records
  // instead of two (header + body) per 16 KiB record.
  SSL_CTX_set_read_ahead(ctx_, 1);
  SSL_CTX_set_default_read_buffer_len(ctx_, 256 * 1024);
  if (verify) {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_PEER, nullptr);
    SSL_CTX_set_default_verify_paths(ctx_);
    if (!ca_file.empty() && SSL_CTX_load_verify_locations(ctx_, ca_file.c_str(), nullptr) != 1) {
      SSL_CTX_free(ctx_);
      ERR_clear_error();
      throw std::runtime_error("cannot load CA file " + ca_file);
    }
  } else {
    SSL_CTX_set_verify(ctx_, SSL_VERIFY_NONE, nullptr);
  }
}

TlsContext::~TlsContext() { SSL_CTX_free(ctx_); }

std::string tls_error(SSL* s, int r, const std::string& what) {
  const int e = SSL_get_error(s, r);
  const int saved = errno;
  unsigned long q = ERR_get_error();
  ERR_clear_error();
  if (q) {
    char buf[256];
    ERR_error_string_n(q, buf, sizeof(buf));
    return what + ": " + buf;
  }
  if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE) return what + " timeout";
  if (e == SSL_ERROR_ZERO_RETURN) return what + ": connection closed";
  if (e == SSL_ERROR_SYSCALL)
    return saved ? what + ": " + strerror(saved) : what + ": unexpected EOF";
  return what + ": SSL error " + std::to_string(e);
}

SSL* tls_handshake(TlsContext& ctx, int fd, const std::string& name) {
  SSL* s = SSL_new(ctx.ctx());
  if (!s) throw std::runtime_error("SSL_new failed");
  SSL_set_fd(s, fd);
  in_addr a4;
  in6_addr a6;
  const bool ip = inet_pton(AF_INET, name.c_str(), &a4) == 1 ||
                  inet_pton(AF_INET6, name.c_str(), &a6) == 1;
  if (!ip) SSL_set_tlsext_host_name(s, name.c_str());  // SNI is for DNS names only
  if (ctx.verify()) {
    X509_VERIFY_PARAM* p = SSL_get0_param(s);
    if (ip)
      X509_VERIFY_PARAM_set1_ip_asc(p, name.c_str());
    else
      SSL_set1_host(s, name.c_str());
  }
  ERR_clear_error();
  const int r = SSL_connect(s);
  if (r != 1) {
    std::string msg = "TLS handshake with " + name;
    const long vr = SSL_get_verify_result(s);
    if (ctx.verify() && vr != X509_V_OK) {
      ERR_clear_error();
      msg += ": certificate verify failed: " + std::string(X509_verify_cert_error_string(vr));
    } else {
      msg = tls_error(s, r, msg);
    }
    SSL_free(s);
    throw std::runtime_error(msg);
  }
  return s;
}

}  // namespace stager
