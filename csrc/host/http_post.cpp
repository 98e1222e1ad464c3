// One HTTP/1.1 POST over a plain TCP socket, for the report sinks
// (report/http.py: Lightning appends, twtml-web stats).
//
// The Python side calls this with the GIL released for the WHOLE exchange.
// Through requests/urllib3 the reporting thread drops and re-takes the GIL
// around every socket call of a request; CPython gives no fairness to a
// waiting thread against a holder that re-takes it quickly, and the
// training thread measured up to ~9 ms stalls behind a 400 KB plot append
// (tools/diag/plot_stall.py).  Connection: close -- one connection per
// request, no pool to guard; responses with Content-Length, chunked, or
// read-to-close bodies.
#include "http_post.h"

#include <charconv>
#include <climits>
#include <cstdint>

#include <netdb.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>
#include <fcntl.h>

#include <algorithm>
#include <cerrno>
#include <chrono>
#include <cstring>
#include <stdexcept>

namespace twtml {
namespace {

using Clock = std::chrono::steady_clock;

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

[[noreturn]] void fail(const std::string& what, int err = 0) {
  throw HttpError(what + (err ? std::string(": ") + std::strerror(err) : std::string()));
}

int remaining_ms(Clock::time_point deadline) {
  const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(deadline - Clock::now()).count();
  return ms > 0 ? int(ms) : 0;
}

void wait_fd(int fd, short ev, Clock::time_point deadline, const char* what) {
  for (;;) {
    pollfd p{fd, ev, 0};
    const int r = ::poll(&p, 1, remaining_ms(deadline));
    if (r > 0) return;
    if (r == 0) fail(std::string("timed out ") + what);
    if (errno != EINTR) fail(std::string("poll ") + what, errno);
  }
}

int connect_to(const std::string& host, int port, Clock::time_point deadline) {
  addrinfo hints{};
  hints.ai_family = AF_UNSPEC;
  hints.ai_socktype = SOCK_STREAM;
  addrinfo* res = nullptr;
  const std::string svc = std::to_string(port);
  const int gai = ::getaddrinfo(host.c_str(), svc.c_str(), &hints, &res);
  if (gai != 0) fail("resolve " + host + ": " + gai_strerror(gai));
  int last_err = 0;
  for (addrinfo* a = res; a; a = a->ai_next) {
    const int fd = ::socket(a->ai_family, a->ai_socktype | SOCK_CLOEXEC | SOCK_NONBLOCK, a->ai_protocol);
    if (fd < 0) {
      last_err = errno;
      continue;
    }
    if (::connect(fd, a->ai_addr, a->ai_addrlen) == 0) {
      ::freeaddrinfo(res);
      return fd;
    }
    if (errno == EINPROGRESS) {
      pollfd p{fd, POLLOUT, 0};
      const int r = ::poll(&p, 1, remaining_ms(deadline));
      int soerr = 0;
      socklen_t len = sizeof(soerr);
      if (r > 0 && ::getsockopt(fd, SOL_SOCKET, SO_ERROR, &soerr, &len) == 0 && soerr == 0) {
        ::freeaddrinfo(res);
        return fd;
      }
      last_err = r == 0 ? ETIMEDOUT : (soerr ? soerr : errno);
    } else {
      last_err = errno;
    }
    ::close(fd);
  }
  ::freeaddrinfo(res);
  fail("connect " + host + ":" + svc, last_err);
}

void send_all(int fd, const char* p, size_t n, Clock::time_point deadline) {
  while (n > 0) {
    const ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w > 0) {
      p += w;
      n -= size_t(w);
    } else if (w < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      wait_fd(fd, POLLOUT, deadline, "sending");
    } else if (w < 0 && errno == EINTR) {
      continue;
    } else {
      fail("send", errno);
    }
  }
}

// the bytes read so far; false at EOF
bool recv_more(int fd, std::string& buf, Clock::time_point deadline) {
  char tmp[16384];
  for (;;) {
    const ssize_t r = ::recv(fd, tmp, sizeof(tmp), 0);
    if (r > 0) {
      buf.append(tmp, size_t(r));
      return true;
    }
    if (r == 0) return false;
    if (errno == EAGAIN || errno == EWOULDBLOCK) {
      wait_fd(fd, POLLIN, deadline, "waiting for the response");
    } else if (errno != EINTR) {
      fail("recv", errno);
    }
  }
}

std::string lower(std::string s) {
  for (auto& c : s) c = char(c >= 'A' && c <= 'Z' ? c - 'A' + 'a' : c);
  return s;
}

// A header number (decimal Content-Length, hex chunk size, optional chunk
// extensions after ';'): malformed or out-of-range text is an HttpError
// (-> requests.ConnectionError in report/http.py), never std::invalid_argument.
uint64_t parse_number(const std::string& text, int base, const char* what) {
  size_t b = text.find_first_not_of(" \t");
  size_t e = text.find_first_of(base == 16 ? "; \t" : " \t", b == std::string::npos ? 0 : b);
  if (b == std::string::npos) b = e = text.size();
  if (e == std::string::npos) e = text.size();
  uint64_t v = 0;
  const auto r = std::from_chars(text.data() + b, text.data() + e, v, base);
  if (b == e || r.ec != std::errc() || r.ptr != text.data() + e) fail(std::string("malformed ") + what + ": '" +
                                                                          text.substr(0, 40) + "'");
  return v;
}

std::string dechunk(const std::string& in) {
  std::string out;
  size_t i = 0;
  for (;;) {
    const size_t eol = in.find("\r\n", i);
    if (eol == std::string::npos) fail("truncated chunked body");
    const uint64_t n = parse_number(in.substr(i, eol - i), 16, "chunk size");
    i = eol + 2;
    if (n == 0) return out;
    if (n > in.size() || i + n > in.size()) fail("truncated chunked body");
    out.append(in, i, n);
    i += n + 2;
  }
}

}  // namespace

HttpResponse http_post(const std::string& host, int port, const std::string& path, const std::string& body,
                       const std::string& extra_headers, double timeout_s) {
  const auto deadline = Clock::now() + std::chrono::microseconds(int64_t(timeout_s * 1e6));
  Fd sock;
  sock.fd = connect_to(host, port, deadline);
  std::string req;
  req.reserve(256 + body.size());
  // an IPv6 literal goes in brackets in the Host header (RFC 7230 5.4)
  const bool v6 = host.find(':') != std::string::npos && host.front() != '[';
  req += "POST " + path + " HTTP/1.1\r\nHost: " + (v6 ? "[" + host + "]" : host) + ":" + std::to_string(port) +
         "\r\nContent-Type: application/json\r\nAccept: application/json\r\nConnection: close\r\n"
         "Content-Length: " + std::to_string(body.size()) + "\r\n" + extra_headers + "\r\n";
  req += body;
  send_all(sock.fd, req.data(), req.size(), deadline);

  std::string buf;
  size_t hdr_end = std::string::npos;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    if (!recv_more(sock.fd, buf, deadline)) fail("connection closed before the response headers");
  }
  HttpResponse res;
  const std::string head = buf.substr(0, hdr_end);
  const size_t sp = head.find(' ');
  if (head.compare(0, 5, "HTTP/") != 0 || sp == std::string::npos) fail("malformed status line");
  res.status = std::atoi(head.c_str() + sp + 1);
  int64_t content_length = -1;
  bool chunked = false;
  for (size_t i = head.find("\r\n"); i != std::string::npos && i < head.size();) {
    const size_t s = i + 2, e = std::min(head.find("\r\n", s), head.size());
    const std::string line = head.substr(s, e - s);
    const size_t c = line.find(':');
    if (c != std::string::npos) {
      const std::string k = lower(line.substr(0, c));
      std::string v = line.substr(c + 1);
      v.erase(0, v.find_first_not_of(" \t"));
      if (k == "content-length") {
        const uint64_t n = parse_number(v, 10, "Content-Length");
        if (n > uint64_t(INT64_MAX)) fail("Content-Length out of range");
        content_length = int64_t(n);
      }
      if (k == "transfer-encoding" && lower(v).find("chunked") != std::string::npos) chunked = true;
    }
    i = e < head.size() ? e : std::string::npos;
  }
  std::string rest = buf.substr(hdr_end + 4);
  if (chunked) {   // Connection: close -- the server closes after the last chunk
    while (recv_more(sock.fd, rest, deadline)) {
    }
    res.body = dechunk(rest);
  } else if (content_length >= 0) {
    while (int64_t(rest.size()) < content_length) {
      if (!recv_more(sock.fd, rest, deadline)) fail("connection closed inside the response body");
    }
    rest.resize(size_t(content_length));
    res.body = std::move(rest);
  } else {
    while (recv_more(sock.fd, rest, deadline)) {
    }
    res.body = std::move(rest);
  }
  return res;
}

}  // namespace twtml
