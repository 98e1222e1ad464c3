// Plain-HTTP POST for the report sinks, run without the GIL (http_post.cpp).
#pragma once

#include <stdexcept>
#include <string>

namespace twtml {

struct HttpResponse {
  int status = 0;
  std::string body;
};

// connection / protocol failures (an HTTP error status is a response)
struct HttpError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// POST body (application/json) to http://host:port/path; extra_headers are
// complete "Name: value\r\n" lines.  The whole exchange within timeout_s.
HttpResponse http_post(const std::string& host, int port, const std::string& path, const std::string& body,
                       const std::string& extra_headers, double timeout_s);

}  // namespace twtml
