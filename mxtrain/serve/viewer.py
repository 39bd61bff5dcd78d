"""Mask R-CNN inspection server -- the single-node replacement of the reference's
"testing" charts (maskrcnn-jupyter / maskrcnn-optimized-jupyter: Jupyter notebook on 1 GPU
running the visualisation notebook, TensorBoard on the train_log, nginx with TLS +
basic auth).

    python -m mxtrain.serve.viewer --logdir /fsx/<log_dir> --port 8888 [--mode predict|metrics]
        [--data-dir /fsx/data/coco2017] [--certfile c.crt --keyfile c.key] [--htpasswd f --user u]

mode predict (the notebook):   GET /             newest checkpoint, links
                               GET /predict[?image=<path>]   PNG overlay (boxes, masks, score>=0.7)
                               GET /predict.json[?image=...] the detections as JSON
mode metrics (TensorBoard):    GET /             stats.json (COCO mAP per epoch) + training
                                                 metrics JSONL as tables
                               GET /stats.json   raw
Both modes: TLS (--certfile/--keyfile) and HTTP basic auth (--htpasswd with
`user:{SHA}base64` or `user:plaintext` lines, like the nginx front-end).  Fail-closed: a
--certfile / --keyfile / --htpasswd that is given but missing (or an htpasswd with no
users) stops the server instead of silently serving plain HTTP or no auth (``--tls off``
and ``--insecure-no-auth`` are the explicit opt-outs; the latter is refused on a
non-loopback bind address), and ``?image=`` only opens files under --data-dir.
"""
from __future__ import annotations

import argparse
import base64
import glob
import hashlib
import html
import io
import json
import os
import random
import ssl
import sys
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer


class ConfigError(SystemExit):
    pass


def load_users(path):
    users = {}
    for line in open(path):
        line = line.strip()
        if ":" in line:
            u, h = line.split(":", 1)
            if u and h:
                users[u] = h
    return users


def safe_image_path(data_dir: str, img: str) -> str:
    """realpath of a requested image, which must lie under realpath(data_dir)."""
    root = os.path.realpath(data_dir)
    cand = os.path.realpath(img if os.path.isabs(img) else os.path.join(root, img))
    if os.path.commonpath([root, cand]) != root:
        raise PermissionError(f"image outside the data directory: {img}")
    if not os.path.isfile(cand):
        raise FileNotFoundError(img)
    return cand


class State:
    def __init__(self, args):
        self.args = args
        self.model = None
        self.ckpt = None
        self.lock = threading.Lock()
        self.users = {}
        if args.htpasswd:
            if not os.path.isfile(args.htpasswd):
                raise ConfigError(f"--htpasswd {args.htpasswd} does not exist (refusing to serve without auth)")
            self.users = load_users(args.htpasswd)
            if not self.users:
                raise ConfigError(f"--htpasswd {args.htpasswd} holds no user:hash line")
        elif not getattr(args, "insecure_no_auth", False):
            raise ConfigError("no --htpasswd given: pass one, or --insecure-no-auth for a loopback-only viewer")
        elif args.host not in ("127.0.0.1", "localhost", "::1"):
            raise ConfigError(f"--insecure-no-auth is only allowed on a loopback address, not {args.host}")

    def check_auth(self, header) -> bool:
        if not self.users:
            return True
        if not header or not header.startswith("Basic "):
            return False
        try:
            u, p = base64.b64decode(header[6:]).decode().split(":", 1)
        except Exception:  # noqa: BLE001
            return False
        h = self.users.get(u)
        if h is None:
            return False
        if h.startswith("{SHA}"):
            return base64.b64encode(hashlib.sha1(p.encode()).digest()).decode() == h[5:]
        return h == p

    def ckpt_dir(self):
        from ..predict import _find_ckpt_dir
        return _find_ckpt_dir(self.args.logdir)

    def load_model(self):
        import torch
        from ..models.maskrcnn import MaskRCNN
        from ..workloads.maskrcnn import config as C
        from ..workloads.maskrcnn.train import latest_ckpt, load_ckpt
        d = self.ckpt_dir()
        ck = latest_ckpt(d)
        if self.model is None or ck != self.ckpt:
            cfg = C.make_config(self.args.config)
            C.finalize(cfg, 1)
            dev = torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")
            m = MaskRCNN(C.model_config(cfg)).to(dev)
            load_ckpt(m, ck)
            self.model, self.ckpt, self.cfg, self.dev = m.eval(), ck, cfg, dev
        return self.model


def make_handler(st: State):
    class H(BaseHTTPRequestHandler):
        def log_message(self, fmt, *a):
            sys.stderr.write("[viewer] " + fmt % a + "\n")

        def _send(self, code, body: bytes, ctype="text/html; charset=utf-8"):
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)

        def do_GET(self):  # noqa: N802
            if not st.check_auth(self.headers.get("Authorization")):
                self.send_response(401)
                self.send_header("WWW-Authenticate", 'Basic realm="mxtrain"')
                self.end_headers()
                return
            u = urllib.parse.urlparse(self.path)
            q = urllib.parse.parse_qs(u.query)
            try:
                if u.path == "/healthz":
                    return self._send(200, b"ok", "text/plain")
                if st.args.mode == "metrics":
                    return self.metrics(u.path)
                return self.predict(u.path, q)
            except PermissionError as e:
                return self._send(403, html.escape(str(e)).encode())
            except FileNotFoundError as e:
                return self._send(404, html.escape(str(e)).encode())
            except Exception as e:  # noqa: BLE001
                return self._send(500, html.escape(repr(e)).encode())

        def metrics(self, path):
            stats = []
            for p in glob.glob(os.path.join(st.args.logdir, "**", "stats.json"), recursive=True):
                stats += json.load(open(p))
            if path == "/stats.json":
                return self._send(200, json.dumps(stats).encode(), "application/json")
            rows = "".join("<tr>" + "".join(f"<td>{html.escape(str(r.get(k, '')))}</td>" for k in sorted(r)) + "</tr>"
                           for r in stats)
            head = "".join(f"<th>{html.escape(k)}</th>" for k in sorted(stats[0])) if stats else ""
            jl = []
            for p in sorted(glob.glob(os.path.join(st.args.logdir, "**", "*.jsonl"), recursive=True))[:8]:
                lines = open(p).read().splitlines()[-20:]
                jl.append(f"<h3>{html.escape(p)}</h3><pre>{html.escape(chr(10).join(lines))}</pre>")
            body = (f"<html><body><h2>mxtrain metrics: {html.escape(st.args.logdir)}</h2>"
                    f"<table border=1><tr>{head}</tr>{rows}</table>{''.join(jl)}</body></html>")
            return self._send(200, body.encode())

        def predict(self, path, q):
            if path == "/":
                d = st.ckpt_dir()
                cks = sorted(glob.glob(os.path.join(d, "model-*.index")))
                body = (f"<html><body><h2>Mask R-CNN checkpoints in {html.escape(d)}</h2><ul>"
                        + "".join(f"<li>{html.escape(os.path.basename(c))}</li>" for c in cks)
                        + "</ul><a href='/predict'>predict a random test2017 image</a></body></html>")
                return self._send(200, body.encode())
            if path in ("/predict", "/predict.json"):
                import tempfile
                from ..predict import predict_images
                img = (q.get("image") or [None])[0]
                if img:
                    img = safe_image_path(st.args.data_dir, img)
                else:
                    c = sorted(glob.glob(os.path.join(st.args.data_dir, "test2017", "*.jpg")))
                    if not c:
                        raise FileNotFoundError(f"no test2017 images under {st.args.data_dir}")
                    img = random.choice(c)
                with st.lock:
                    m = st.load_model()
                    out = tempfile.mkdtemp(prefix="viewer-")
                    rec = predict_images(m, [img], st.dev, out, st.cfg.PREPROC.TRAIN_SHORT,
                                         int(st.cfg.PREPROC.MAX_SIZE), st.args.score_thresh,
                                         st.args.mask_thresh)[0]
                if path == "/predict.json":
                    return self._send(200, json.dumps(rec).encode(), "application/json")
                return self._send(200, open(rec["output"], "rb").read(), "image/png")
            return self._send(404, b"not found")
    return H


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--port", type=int, default=8888)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--mode", default="predict", choices=["predict", "metrics"])
    ap.add_argument("--data-dir", default="/fsx/data/coco2017")
    ap.add_argument("--score-thresh", type=float, default=0.7)
    ap.add_argument("--mask-thresh", type=float, default=0.5)
    ap.add_argument("--certfile", default=None)
    ap.add_argument("--keyfile", default=None)
    ap.add_argument("--tls", default="auto", choices=["auto", "off"],
                    help="auto: TLS when --certfile/--keyfile are given (they must exist); off: plain HTTP")
    ap.add_argument("--htpasswd", default=None)
    ap.add_argument("--insecure-no-auth", action="store_true",
                    help="serve without basic auth (loopback bind addresses only)")
    ap.add_argument("--config", nargs="*", default=[])
    a = ap.parse_args(argv)
    try:
        st = State(a)
        ctx = None
        if a.tls != "off" and (a.certfile or a.keyfile):
            for f in (a.certfile, a.keyfile):
                if not f or not os.path.isfile(f):
                    raise ConfigError(f"TLS certificate/key {f!r} missing (use --tls off to serve plain HTTP)")
            ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
            ctx.load_cert_chain(a.certfile, a.keyfile)
    except ConfigError as e:
        print(f"[viewer] refusing to start: {e}", file=sys.stderr, flush=True)
        return 2
    srv = ThreadingHTTPServer((a.host, a.port), make_handler(st))
    if ctx is not None:
        srv.socket = ctx.wrap_socket(srv.socket, server_side=True)
    print(f"[viewer] serving {a.mode} for {a.logdir} on {a.host}:{a.port} "
          f"({'https' if ctx else 'http'}, basic auth {'on' if st.users else 'OFF (loopback)'})", flush=True)
    srv.serve_forever()


if __name__ == "__main__":
    sys.exit(main())
