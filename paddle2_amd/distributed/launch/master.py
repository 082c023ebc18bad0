"""HTTP key-value master for launcher rendezvous (``--master http://host:port``).

Reference behaviour: python/paddle/distributed/launch/controllers/master.py ``HTTPMaster.sync_peers`` over
launch/utils/kv_server.py / kv_client.py — one node hosts a small HTTP key-value service, every node PUTs its
descriptor under ``prefix/key/rank`` and polls the prefix until ``size`` descriptors are present; the sorted
descriptor list and this node's position in it are the node ranks.

Design here: a stdlib ``ThreadingHTTPServer`` holding one dict behind a lock (the reference's server is the same
shape), JSON for prefix listings, and a client with bounded retries.  The default rendezvous of the launcher stays
the native TCPStore (csrc/runtime/tcp_store.cpp); this master is the reference-compatible alternative for
clusters that expose only HTTP between nodes.

Routes::

    PUT    /kv/<key>          body = value bytes        -> 200
    GET    /kv/<key>                                    -> 200 value | 404
    DELETE /kv/<key>                                    -> 200
    GET    /prefix/<prefix>                             -> 200 {"key": "value (latin-1)", ...}
    GET    /healthz                                     -> 200 "ok"
"""
from __future__ import annotations

import json
import threading
import time
import urllib.error
import urllib.parse
import urllib.request
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class _Handler(BaseHTTPRequestHandler):
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # quiet: launcher logs are the worker logs
        pass

    def _reply(self, code, body=b"", ctype="application/octet-stream"):
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        if body:
            self.wfile.write(body)

    def _key(self, head):
        return urllib.parse.unquote(self.path[len(head):])

    def do_GET(self):  # noqa: N802 (http.server naming)
        kv, lock = self.server.kv, self.server.lock
        if self.path == "/healthz":
            return self._reply(200, b"ok", "text/plain")
        if self.path.startswith("/kv/"):
            with lock:
                v = kv.get(self._key("/kv/"))
            return self._reply(404) if v is None else self._reply(200, v)
        if self.path.startswith("/prefix/"):
            p = self._key("/prefix/")
            with lock:
                out = {k: v.decode("latin-1") for k, v in kv.items() if k.startswith(p)}
            return self._reply(200, json.dumps(out).encode(), "application/json")
        return self._reply(404)

    def do_PUT(self):  # noqa: N802
        if not self.path.startswith("/kv/"):
            return self._reply(404)
        n = int(self.headers.get("Content-Length", "0"))
        v = self.rfile.read(n) if n else b""
        with self.server.lock:
            self.server.kv[self._key("/kv/")] = v
        return self._reply(200)

    def do_DELETE(self):  # noqa: N802
        if not self.path.startswith("/kv/"):
            return self._reply(404)
        with self.server.lock:
            self.server.kv.pop(self._key("/kv/"), None)
        return self._reply(200)


class KVServer:
    """The HTTP key-value service (reference launch/utils/kv_server.py KVServer)."""

    def __init__(self, port, host="0.0.0.0"):
        self.httpd = ThreadingHTTPServer((host, int(port)), _Handler)
        self.httpd.daemon_threads = True
        self.httpd.kv = {}
        self.httpd.lock = threading.Lock()
        self.port = self.httpd.server_address[1]
        self._th = None
        self.started = False
        self.stopped = False

    def start(self):
        if not self.started:
            self._th = threading.Thread(target=self.httpd.serve_forever, kwargs={"poll_interval": 0.1}, daemon=True)
            self._th.start()
            self.started = True

    def stop(self):
        if self.started and not self.stopped:
            self.httpd.shutdown()
            self.httpd.server_close()
            self._th.join(timeout=5)
            self.stopped = True


class KVClient:
    """Client of a KVServer (reference launch/utils/kv_client.py): methods return False / None on failure."""

    def __init__(self, endpoint, timeout=5.0):
        ep = endpoint[len("http://"):] if endpoint.startswith("http://") else endpoint
        self.base = f"http://{ep}"
        self.timeout = timeout

    def _req(self, method, path, data=None):
        req = urllib.request.Request(self.base + path, data=data, method=method)
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as r:
                return r.status, r.read()
        except urllib.error.HTTPError as e:
            return e.code, b""
        except (urllib.error.URLError, OSError):
            return None, b""

    def put(self, key, value):
        if isinstance(value, str):
            value = value.encode()
        code, _ = self._req("PUT", "/kv/" + urllib.parse.quote(key, safe=""), value)
        return code == 200

    def get(self, key):
        code, body = self._req("GET", "/kv/" + urllib.parse.quote(key, safe=""))
        return body if code == 200 else None

    def delete(self, key):
        code, _ = self._req("DELETE", "/kv/" + urllib.parse.quote(key, safe=""))
        return code == 200

    def get_prefix(self, prefix):
        code, body = self._req("GET", "/prefix/" + urllib.parse.quote(prefix, safe=""))
        return json.loads(body) if code == 200 else None

    def wait_server_ready(self, timeout=3.0):
        end = time.time() + timeout
        while time.time() < end:
            code, body = self._req("GET", "/healthz")
            if code == 200 and body == b"ok":
                return True
            time.sleep(0.05)
        return False


class HTTPMaster:
    """Rendezvous over a KVServer.  ``endpoint`` "host:port"; the node that can bind it (or ``is_main``) hosts the
    server.  ``sync_peers`` returns (the sorted peer values, this node's index)."""

    def __init__(self, endpoint, is_main=None, timeout=600.0):
        ep = endpoint[len("http://"):] if endpoint.startswith("http://") else endpoint
        self.endpoint = ep
        host, port = ep.rsplit(":", 1)
        self.server = None
        if is_main is None or is_main:
            try:
                self.server = KVServer(int(port), host="0.0.0.0")
                self.server.start()
            except OSError:
                if is_main:
                    raise
                self.server = None   # another node hosts it
        self.is_main = self.server is not None
        self.client = KVClient(ep)
        self.timeout = timeout

    def sync_peers(self, prefix, key, value, size, rank=-1):
        """Publish ``value`` under ``prefix/<key>/<rank>`` and wait for ``size`` peers.  Order: by explicit rank
        when every peer gave one, else by key with the hosting node first (the reference's 'aaaaaa' key)."""
        if size < 2:
            return [value], 0
        deadline = time.time() + self.timeout
        while not self.client.wait_server_ready(timeout=5.0):
            if time.time() > deadline:
                raise TimeoutError(f"HTTP master {self.endpoint} not reachable")
        ky = "aaaaaa" if (rank < 0 and self.is_main) else key
        me = f"{prefix}/{ky}/{rank}"
        while not self.client.put(me, value):
            if time.time() > deadline:
                raise TimeoutError("HTTP master: put failed")
            time.sleep(0.1)
        while True:
            got = self.client.get_prefix(prefix + "/")
            if got is not None and len(got) >= size:
                break
            if time.time() > deadline:
                raise TimeoutError(f"HTTP master: {0 if got is None else len(got)} of {size} peers")
            time.sleep(0.1)
        if all(k.rsplit("/", 1)[1] not in ("-1", "") for k in got):
            keys = sorted(got, key=lambda k: int(k.rsplit("/", 1)[1]))
        else:
            keys = sorted(got)
        keys = keys[:size]
        return [got[k] for k in keys], keys.index(me)

    def stop(self, linger=2.0):
        """Stop the hosted server — after ``linger`` seconds, so peers still polling the prefix see the full set."""
        if self.server is not None:
            time.sleep(linger)
            self.server.stop()
