"""Built-in log viewer (the role of the kubernetes-dashboard / tf-job-dashboard URLs that
``arena logviewer`` prints in the reference: dashboard_helper.go:12-47, trainer_mpi.go:34-63,
trainer_tensorflow.go:106-133; the reference deploys kubernetes/dashboard/dashboard.yaml:1-104).

Runs against either backend: the local job store (started on demand by ``arena logviewer``), or a
cluster -- ``deploy/logviewer.yaml`` runs it as the ``kubernetes-dashboard`` Deployment + Service in
``arena-system`` with ``--backend k8s``, reading pod logs through the API server with its service
account, so ``arena logviewer <job>`` on the K8s backend resolves that Service's Endpoints.

Serves the same URL shapes the CLI prints, so they work unchanged:
  http://<node>:<port>/#!/log/<ns>/<pod>/<container>?namespace=<ns>   (MPI / standalone)
  http://<node>:<port>/tfjobs/ui/#/<ns>/<tfjob>                      (PS/worker)
plus a job index at ``/``. The fragment is resolved client-side; data comes from
``/api/jobs`` and ``/api/log/<ns>/<pod>?tail=N`` (read from the job store, never the GPU).

    python -m arena_amd.runtime.logviewer --home ~/.arena --port 0
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import parse_qs, unquote, urlparse

PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>arena log viewer</title>
<style>body{font-family:sans-serif;margin:1.5em}pre{background:#111;color:#ddd;padding:1em;
white-space:pre-wrap;max-height:80vh;overflow:auto}td,th{padding:2px 10px;text-align:left}</style>
</head><body><h2 id="title">arena jobs</h2><div id="main">loading...</div><script>
async function jobs(){return (await fetch('/api/jobs')).json();}
function esc(s){return s.replace(/[&<>]/g,c=>({'&':'&amp;','<':'&lt;','>':'&gt;'}[c]));}
async function showLog(ns,pod){
  document.getElementById('title').textContent='log: '+pod;
  const r=await fetch('/api/log/'+ns+'/'+pod+'?tail=2000');
  document.getElementById('main').innerHTML='<pre>'+esc(await r.text())+'</pre>';
  setTimeout(()=>route(),2000);}
function podLink(ns,p){return '<a href="#!/log/'+ns+'/'+p.name+'/'+p.container+'?namespace='+ns+'">'+p.name+'</a>';}
async function showJobs(filterNs,filterName){
  const js=await jobs();let h='<table><tr><th>job</th><th>namespace</th><th>status</th><th>pods</th></tr>';
  for(const j of js){ if(filterName && !(filterName===j.name||filterName.startsWith(j.name+'-'))) continue;
    h+='<tr><td>'+j.name+'</td><td>'+j.namespace+'</td><td>'+j.status+'</td><td>'+
       j.pods.map(p=>podLink(j.namespace,p)+' ('+p.phase+')').join('<br>')+'</td></tr>';}
  document.getElementById('main').innerHTML=h+'</table>';}
function route(){const h=decodeURIComponent(location.hash);let m;
  if((m=h.match(/^#!\\/log\\/([^/]+)\\/([^/?]+)/))) return showLog(m[1],m[2]);
  if((m=h.match(/^#\\/([^/]+)\\/([^/?]+)/))) return showJobs(m[1],m[2]);
  document.getElementById('title').textContent='arena jobs'; return showJobs();}
window.onhashchange=route; route();
</script></body></html>"""


def make_handler(backend):
    from ..jobs.trainer import get_training_job

    class H(BaseHTTPRequestHandler):
        def log_message(self, *a):  # quiet
            pass

        def _send(self, code, body, ctype):
            data = body.encode() if isinstance(body, str) else body
            self.send_response(code)
            self.send_header("Content-Type", ctype)
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):  # noqa: N802
            u = urlparse(self.path)
            if u.path in ("/", "/index.html") or u.path.startswith("/tfjobs/ui"):
                return self._send(200, PAGE, "text/html; charset=utf-8")
            if u.path == "/api/jobs":
                out = []
                for name, ns in sorted(backend.list_releases().items()):
                    pods = backend.list_pods(ns, {"release": name})
                    try:
                        st = get_training_job(backend, name, ns).get_status() or "Unknown"
                    except Exception:  # noqa: BLE001 - a job being deleted: still list it
                        st = "Unknown"
                    out.append({"name": name, "namespace": ns, "status": st,
                                "pods": [{"name": p.name, "phase": p.phase,
                                          "container": p.containers[0].name if p.containers else ""}
                                         for p in sorted(pods, key=lambda p: p.name)]})
                return self._send(200, json.dumps(out), "application/json")
            if u.path.startswith("/api/log/"):
                parts = [unquote(x) for x in u.path[len("/api/log/"):].split("/")]
                if len(parts) < 2:
                    return self._send(400, "bad path", "text/plain")
                tail = int(parse_qs(u.query).get("tail", ["-1"])[0])
                try:
                    text = "".join(backend.pod_logs(parts[0], parts[1], tail=tail))
                except Exception as e:  # noqa: BLE001
                    return self._send(404, str(e), "text/plain")
                return self._send(200, text, "text/plain; charset=utf-8")
            return self._send(404, "not found", "text/plain")
    return H


def serve(backend, host: str = "0.0.0.0", port: int = 0, ready_file: str = "") -> None:
    srv = ThreadingHTTPServer((host, port), make_handler(backend))
    if ready_file:
        tmp = ready_file + ".tmp"
        with open(tmp, "w") as f:
            json.dump({"pid": os.getpid(), "port": srv.server_address[1]}, f)
        os.replace(tmp, ready_file)
    print(f"arena log viewer on http://{host}:{srv.server_address[1]}/", flush=True)
    srv.serve_forever()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="arena log viewer")
    ap.add_argument("--home", default=os.environ.get("ARENA_HOME",
                                                     os.path.join(os.path.expanduser("~"), ".arena")))
    ap.add_argument("--backend", choices=["local", "k8s"],
                    default=os.environ.get("ARENA_BACKEND", "local"))
    ap.add_argument("--config", default=os.environ.get("KUBECONFIG", ""),
                    help="kubeconfig (k8s backend; in a pod the service account is used)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=0)
    ap.add_argument("--ready-file", default="")
    a = ap.parse_args(argv)
    if a.backend == "k8s":
        from ..cluster.k8s import K8sBackend
        backend = K8sBackend(kubeconfig=a.config, home=a.home)
    else:
        from ..cluster.local import LocalBackend
        backend = LocalBackend(a.home)
    serve(backend, a.host, a.port, a.ready_file)
    return 0


if __name__ == "__main__":
    sys.exit(main())
