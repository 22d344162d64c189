"""Probe: is kernel TLS (TCP_ULP "tls") available to this user? Prints the kernel, whether
the tls ULP attaches to a connected loopback TCP socket, and OpenSSL's version."""
import socket
import ssl
import platform

TCP_ULP = 31
srv = socket.socket()
srv.bind(("127.0.0.1", 0))
srv.listen(1)
c = socket.create_connection(srv.getsockname())
a, _ = srv.accept()
try:
    c.setsockopt(socket.IPPROTO_TCP, TCP_ULP, b"tls")
    ok = "attached"
except OSError as e:
    ok = f"refused: {e}"
print({"kernel": platform.release(), "tls_ulp": ok, "openssl": ssl.OPENSSL_VERSION,
       "avail_ulp": open("/proc/sys/net/ipv4/tcp_available_ulp").read().strip()
       if __import__("os").path.exists("/proc/sys/net/ipv4/tcp_available_ulp") else None})
