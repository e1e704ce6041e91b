"""Built-in TensorBoard-lite: serves the scalars of a log directory over HTTP.

    python -m arena_amd.tb.server --logdir DIR --port 6006

``/`` renders every (run, tag) series as an inline-SVG line chart; ``/data/scalars`` returns JSON.
Used by the local backend for `--tensorboard` (the real `tensorboard` binary is used instead when
it is installed and ``ARENA_USE_TENSORBOARD=1``).
"""
from __future__ import annotations

import argparse
import html
import json
import os
import shutil
import subprocess
import sys
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

from .writer import read_scalars


def _svg(points, w=520, h=180) -> str:
    if not points:
        return ""
    xs = [p[0] for p in points]
    ys = [p[1] for p in points]
    x0, x1 = min(xs), max(xs) or 1
    y0, y1 = min(ys), max(ys)
    if y1 == y0:
        y1 = y0 + 1
    sx = (w - 60) / max(x1 - x0, 1)
    sy = (h - 30) / (y1 - y0)
    pts = " ".join(f"{50 + (x - x0) * sx:.1f},{h - 20 - (y - y0) * sy:.1f}" for x, y in points)
    return (f'<svg width="{w}" height="{h}" style="background:#fafafa;border:1px solid #ddd">'
            f'<polyline fill="none" stroke="#e8710a" stroke-width="1.5" points="{pts}"/>'
            f'<text x="2" y="12" font-size="10">{y1:.4g}</text>'
            f'<text x="2" y="{h - 22}" font-size="10">{y0:.4g}</text>'
            f'<text x="50" y="{h - 4}" font-size="10">step {x0}</text>'
            f'<text x="{w - 80}" y="{h - 4}" font-size="10">step {x1}</text></svg>')


def make_handler(logdir: str):
    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            return

        def _send(self, code, body, ctype):
            data = body.encode()
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):  # noqa: N802
            scal = read_scalars(logdir)
            if self.path.startswith("/data/scalars"):
                self._send(200, json.dumps(scal), "application/json")
                return
            parts = [f"<html><head><title>arena tensorboard</title></head><body>"
                     f"<h2>Scalars: {html.escape(logdir)}</h2>"]
            for run, tags in sorted(scal.items()):
                for tag, pts in sorted(tags.items()):
                    last = pts[-1][1] if pts else float("nan")
                    parts.append(f"<h4>{html.escape(run)} / {html.escape(tag)} "
                                 f"(last {last:.5g})</h4>{_svg(sorted(pts))}")
            if not scal:
                parts.append("<p>No scalar data yet.</p>")
            parts.append("</body></html>")
            self._send(200, "".join(parts), "text/html")

    return H


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--port", type=int, default=6006)
    ap.add_argument("--host", default="0.0.0.0")
    a = ap.parse_args(argv)
    os.makedirs(a.logdir, exist_ok=True)
    if os.environ.get("ARENA_USE_TENSORBOARD") == "1" and shutil.which("tensorboard"):
        return subprocess.call(["tensorboard", "--logdir", a.logdir, "--host", a.host,
                                "--port", str(a.port)])
    srv = ThreadingHTTPServer((a.host, a.port), make_handler(a.logdir))
    print(f"arena tensorboard serving {a.logdir} on http://{a.host}:{a.port}", flush=True)
    try:
        srv.serve_forever()
    except KeyboardInterrupt:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
