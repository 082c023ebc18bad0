// TCPStore: the rendezvous key-value store of the distributed runtime.
//
// Reference behaviour: paddle/phi/core/distributed/store/tcp_store.{h,cc} (MasterDaemon with
// set/get/add/wait/check, a client per rank, used to exchange comm unique ids and to barrier
// during init) and tcp_utils.cc.  This is an independent design: one poll(2) event loop on the
// master serves every client over non-blocking sockets; blocking GET / WAIT requests are parked
// as waiters and answered the moment the awaited keys are set, so the daemon never dedicates a
// thread per client.  Wire format (little endian): request = u8 cmd, then length-prefixed
// fields (u32 len + bytes); replies are u8 status or a length-prefixed value.
#include "runtime.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace pdrt {

enum Cmd : uint8_t { kSet = 1, kGet = 2, kAdd = 3, kCheck = 4, kWait = 5, kDelete = 6, kNumKeys = 7, kCas = 8, kAppend = 9 };

static void put_u32(std::string& b, uint32_t v) { b.append(reinterpret_cast<const char*>(&v), 4); }
static void put_str(std::string& b, const std::string& s) { put_u32(b, (uint32_t)s.size()); b += s; }

// ---------------------------------------------------------------------------------- server
struct TCPStoreServer::Impl {
  int lfd = -1;
  int port = 0;
  std::atomic<bool> stop{false};
  std::thread loop;
  std::unordered_map<std::string, std::string> kv;
  struct Conn {
    int fd;
    std::string in, out;
  };
  struct Waiter {
    int fd;
    uint8_t cmd;
    std::vector<std::string> keys;
  };
  std::vector<Conn> conns;
  std::vector<Waiter> waiters;
  int wake[2] = {-1, -1};

  Conn* find(int fd) {
    for (auto& c : conns)
      if (c.fd == fd) return &c;
    return nullptr;
  }

  bool have_all(const std::vector<std::string>& keys) {
    for (auto& k : keys)
      if (!kv.count(k)) return false;
    return true;
  }

  void reply_waiter(const Waiter& w) {
    Conn* c = find(w.fd);
    if (!c) return;
    if (w.cmd == kGet) put_str(c->out, kv[w.keys[0]]);
    else c->out.push_back(1);
  }

  void wake_waiters() {
    std::vector<Waiter> keep;
    for (auto& w : waiters) {
      if (have_all(w.keys)) reply_waiter(w);
      else keep.push_back(w);
    }
    waiters.swap(keep);
  }

  // parse as many complete requests as the buffer holds; returns false on protocol error
  bool handle(Conn& c) {
    for (;;) {
      size_t p = 0;
      auto need = [&](size_t n) { return c.in.size() >= p + n; };
      auto rd_u32 = [&](uint32_t& v) {
        if (!need(4)) return false;
        std::memcpy(&v, c.in.data() + p, 4);
        p += 4;
        return true;
      };
      auto rd_str = [&](std::string& s) {
        uint32_t n;
        if (!rd_u32(n)) return false;
        if (!need(n)) return false;
        s.assign(c.in.data() + p, n);
        p += n;
        return true;
      };
      if (!need(1)) return true;
      const uint8_t cmd = (uint8_t)c.in[p++];
      std::string k, v, v2;
      bool ok = true;
      switch (cmd) {
        case kSet:
          if (!rd_str(k) || !rd_str(v)) return true;
          kv[k] = v;
          c.out.push_back(1);
          wake_waiters();
          break;
        case kGet:
          if (!rd_str(k)) return true;
          if (kv.count(k)) put_str(c.out, kv[k]);
          else waiters.push_back({c.fd, kGet, {k}});
          break;
        case kAdd: {
          if (!rd_str(k) || !rd_str(v)) return true;
          int64_t inc = 0, cur = 0;
          std::memcpy(&inc, v.data(), std::min<size_t>(8, v.size()));
          auto it = kv.find(k);
          if (it != kv.end()) cur = std::stoll(it->second);
          cur += inc;
          kv[k] = std::to_string(cur);
          c.out.append(reinterpret_cast<const char*>(&cur), 8);
          wake_waiters();
          break;
        }
        case kCheck:
        case kWait: {
          uint32_t n;
          if (!rd_u32(n)) return true;
          std::vector<std::string> keys(n);
          for (auto& kk : keys)
            if (!rd_str(kk)) return true;
          if (cmd == kCheck) c.out.push_back(have_all(keys) ? 1 : 0);
          else if (have_all(keys)) c.out.push_back(1);
          else waiters.push_back({c.fd, kWait, keys});
          break;
        }
        case kDelete:
          if (!rd_str(k)) return true;
          c.out.push_back(kv.erase(k) ? 1 : 0);
          break;
        case kNumKeys: {
          int64_t n = (int64_t)kv.size();
          c.out.append(reinterpret_cast<const char*>(&n), 8);
          break;
        }
        case kAppend: {
          // atomic on the server (one event loop): concurrent appends of identical bytes both land, which a
          // client-side read / compare_set loop cannot guarantee (ABA on equal values); returns the new length
          if (!rd_str(k) || !rd_str(v)) return true;
          std::string& cur = kv[k];
          cur += v;
          const int64_t n = (int64_t)cur.size();
          c.out.append(reinterpret_cast<const char*>(&n), 8);
          wake_waiters();
          break;
        }
        case kCas: {
          if (!rd_str(k) || !rd_str(v) || !rd_str(v2)) return true;
          auto it = kv.find(k);
          if ((it == kv.end() && v.empty()) || (it != kv.end() && it->second == v)) kv[k] = v2;
          put_str(c.out, kv.count(k) ? kv[k] : v);
          wake_waiters();
          break;
        }
        default:
          ok = false;
      }
      if (!ok) return false;
      c.in.erase(0, p);
    }
  }

  void run() {
    while (!stop.load()) {
      std::vector<pollfd> pf;
      pf.push_back({lfd, POLLIN, 0});
      pf.push_back({wake[0], POLLIN, 0});
      for (auto& c : conns) pf.push_back({c.fd, (short)(POLLIN | (c.out.empty() ? 0 : POLLOUT)), 0});
      int r = ::poll(pf.data(), pf.size(), 200);
      if (r <= 0) continue;
      if (pf[0].revents & POLLIN) {
        int fd = ::accept(lfd, nullptr, nullptr);
        if (fd >= 0) {
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          fcntl(fd, F_SETFL, O_NONBLOCK);
          conns.push_back({fd, {}, {}});
        }
      }
      std::vector<int> dead;
      for (size_t i = 2; i < pf.size(); ++i) {
        Conn* c = find(pf[i].fd);
        if (!c) continue;
        if (pf[i].revents & (POLLERR | POLLHUP | POLLNVAL)) {
          dead.push_back(c->fd);
          continue;
        }
        if (pf[i].revents & POLLIN) {
          char buf[65536];
          ssize_t n = ::recv(c->fd, buf, sizeof(buf), 0);
          if (n <= 0) {
            dead.push_back(c->fd);
            continue;
          }
          c->in.append(buf, (size_t)n);
          if (!handle(*c)) {
            dead.push_back(c->fd);
            continue;
          }
        }
      }
      for (auto& c : conns) {
        while (!c.out.empty()) {
          ssize_t n = ::send(c.fd, c.out.data(), c.out.size(), MSG_NOSIGNAL);
          if (n <= 0) break;
          c.out.erase(0, (size_t)n);
        }
      }
      for (int fd : dead) {
        ::close(fd);
        for (size_t i = 0; i < conns.size(); ++i)
          if (conns[i].fd == fd) { conns.erase(conns.begin() + i); break; }
        std::vector<Waiter> keep;
        for (auto& w : waiters)
          if (w.fd != fd) keep.push_back(w);
        waiters.swap(keep);
      }
    }
  }
};

TCPStoreServer::TCPStoreServer(const std::string& host, int port) : impl_(new Impl) {
  impl_->lfd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (impl_->lfd < 0) throw std::runtime_error("TCPStore: socket() failed");
  int one = 1;
  setsockopt(impl_->lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = host.empty() || host == "0.0.0.0" ? INADDR_ANY : inet_addr(host.c_str());
  if (::bind(impl_->lfd, (sockaddr*)&a, sizeof(a)) != 0) {
    ::close(impl_->lfd);
    throw std::runtime_error("TCPStore: bind to port " + std::to_string(port) + " failed: " + strerror(errno));
  }
  socklen_t len = sizeof(a);
  getsockname(impl_->lfd, (sockaddr*)&a, &len);
  impl_->port = ntohs(a.sin_port);
  ::listen(impl_->lfd, 1024);
  if (::pipe(impl_->wake) != 0) throw std::runtime_error("TCPStore: pipe() failed");
  impl_->loop = std::thread([this] { impl_->run(); });
}

TCPStoreServer::~TCPStoreServer() { shutdown(); }

int TCPStoreServer::port() const { return impl_->port; }

void TCPStoreServer::shutdown() {
  if (!impl_ || impl_->stop.exchange(true)) return;
  if (impl_->wake[1] >= 0) (void)!::write(impl_->wake[1], "x", 1);
  if (impl_->loop.joinable()) impl_->loop.join();
  for (auto& c : impl_->conns) ::close(c.fd);
  ::close(impl_->lfd);
  ::close(impl_->wake[0]);
  ::close(impl_->wake[1]);
}

// ---------------------------------------------------------------------------------- client
TCPStoreClient::TCPStoreClient(const std::string& host, int port, double timeout_s) : timeout_s_(timeout_s) {
  auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
  for (;;) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
      if (::connect(fd_, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        break;
      }
      ::close(fd_);
      fd_ = -1;
      freeaddrinfo(res);
    }
    if (std::chrono::steady_clock::now() > deadline)
      throw std::runtime_error("TCPStore: connect to " + host + ":" + std::to_string(port) + " timed out");
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  int one = 1;
  setsockopt(fd_, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  set_timeout(timeout_s);
}

TCPStoreClient::~TCPStoreClient() {
  if (fd_ >= 0) ::close(fd_);
}

void TCPStoreClient::set_timeout(double s) {
  timeout_s_ = s;
  timeval tv{};
  tv.tv_sec = (long)s;
  tv.tv_usec = (long)((s - (long)s) * 1e6);
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
}

void TCPStoreClient::send_all(const std::string& b) {
  size_t off = 0;
  while (off < b.size()) {
    ssize_t n = ::send(fd_, b.data() + off, b.size() - off, MSG_NOSIGNAL);
    if (n <= 0) throw std::runtime_error("TCPStore: send failed");
    off += (size_t)n;
  }
}

void TCPStoreClient::recv_all(char* p, size_t n) {
  size_t off = 0;
  while (off < n) {
    ssize_t r = ::recv(fd_, p + off, n - off, 0);
    if (r <= 0) throw std::runtime_error("TCPStore: receive failed or timed out");
    off += (size_t)r;
  }
}

std::string TCPStoreClient::recv_str() {
  uint32_t n;
  recv_all(reinterpret_cast<char*>(&n), 4);
  std::string s(n, '\0');
  if (n) recv_all(&s[0], n);
  return s;
}

void TCPStoreClient::set(const std::string& k, const std::string& v) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kSet);
  put_str(b, k);
  put_str(b, v);
  send_all(b);
  char ok;
  recv_all(&ok, 1);
}

std::string TCPStoreClient::get(const std::string& k) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kGet);
  put_str(b, k);
  send_all(b);
  return recv_str();
}

int64_t TCPStoreClient::add(const std::string& k, int64_t inc) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kAdd);
  put_str(b, k);
  put_str(b, std::string(reinterpret_cast<const char*>(&inc), 8));
  send_all(b);
  int64_t v;
  recv_all(reinterpret_cast<char*>(&v), 8);
  return v;
}

bool TCPStoreClient::check(const std::vector<std::string>& keys) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kCheck);
  put_u32(b, (uint32_t)keys.size());
  for (auto& k : keys) put_str(b, k);
  send_all(b);
  char ok;
  recv_all(&ok, 1);
  return ok != 0;
}

void TCPStoreClient::wait(const std::vector<std::string>& keys) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kWait);
  put_u32(b, (uint32_t)keys.size());
  for (auto& k : keys) put_str(b, k);
  send_all(b);
  char ok;
  recv_all(&ok, 1);
}

bool TCPStoreClient::remove(const std::string& k) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kDelete);
  put_str(b, k);
  send_all(b);
  char ok;
  recv_all(&ok, 1);
  return ok != 0;
}

int64_t TCPStoreClient::num_keys() {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kNumKeys);
  send_all(b);
  int64_t v;
  recv_all(reinterpret_cast<char*>(&v), 8);
  return v;
}

int64_t TCPStoreClient::append(const std::string& k, const std::string& v) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kAppend);
  put_str(b, k);
  put_str(b, v);
  send_all(b);
  int64_t n;
  recv_all(reinterpret_cast<char*>(&n), 8);
  return n;
}

std::string TCPStoreClient::compare_set(const std::string& k, const std::string& expected, const std::string& desired) {
  std::lock_guard<std::mutex> g(mu_);
  std::string b(1, (char)kCas);
  put_str(b, k);
  put_str(b, expected);
  put_str(b, desired);
  send_all(b);
  return recv_str();
}

}  // namespace pdrt
