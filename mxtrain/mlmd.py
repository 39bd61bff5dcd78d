"""Pipeline run metadata and lineage (the KFP metadata store, MLMD).

The reference's Kubeflow Pipelines install runs ml-metadata's gRPC store next to the API
server (charts/ml-platform/kubeflow-pipelines/templates/deployments.yaml: metadata-grpc /
metadata-writer) so that every pipeline step becomes an *execution* linked to the
*artifacts* it read and wrote, grouped under *contexts* (the pipeline, the run).  Here the
same data model lives in one SQLite file under ``$MXTRAIN_HOME/pipelines/metadata.db``,
written by ``pipeline.run_pipeline`` as the steps run:

* contexts   -- ``pipeline`` (a stored pipeline definition) and ``run``; a run's parent
               context is its pipeline;
* executions -- one per chart step (``chart_step``): release, namespace, chart, cache key,
               state NEW -> RUNNING -> COMPLETE / FAILED / CANCELED, or CACHED when the step
               cache served it (property ``cached_from``: the execution that produced it);
* artifacts  -- the step's inputs (``Chart``: chart directory + content digest;
               ``ChartValues``: the values override, by digest) and its output
               (``ReleaseRecord``: the release's record directory -- status, manifests,
               pod logs); identical inputs are one artifact shared by every execution that
               read them (KFP dedups by URI + digest the same way);
* events     -- execution <-> artifact edges, INPUT or OUTPUT; attributions /
               associations tie artifacts / executions to contexts.

Queries: ``run_lineage(run)`` (the run's executions with their input / output artifacts)
and ``artifact_lineage(id)`` (the executions that produced and consumed an artifact, and
transitively their inputs) -- served by the dashboard as ``GET /api/runs/<run>/lineage``
and ``GET /api/artifacts/<id>/lineage``.
"""
from __future__ import annotations

import hashlib
import json
import os
import sqlite3
import threading
import time
from contextlib import contextmanager
from typing import Dict, List, Optional

_LOCK = threading.Lock()

_SCHEMA = """
CREATE TABLE IF NOT EXISTS contexts (
  id INTEGER PRIMARY KEY, type TEXT NOT NULL, name TEXT NOT NULL, properties TEXT NOT NULL,
  created REAL NOT NULL, UNIQUE (type, name));
CREATE TABLE IF NOT EXISTS parent_contexts (
  child INTEGER NOT NULL, parent INTEGER NOT NULL, PRIMARY KEY (child, parent));
CREATE TABLE IF NOT EXISTS executions (
  id INTEGER PRIMARY KEY, type TEXT NOT NULL, name TEXT NOT NULL, state TEXT NOT NULL,
  properties TEXT NOT NULL, created REAL NOT NULL, updated REAL NOT NULL);
CREATE TABLE IF NOT EXISTS artifacts (
  id INTEGER PRIMARY KEY, type TEXT NOT NULL, uri TEXT NOT NULL, digest TEXT NOT NULL,
  properties TEXT NOT NULL, created REAL NOT NULL, UNIQUE (type, uri, digest));
CREATE TABLE IF NOT EXISTS events (
  execution INTEGER NOT NULL, artifact INTEGER NOT NULL, type TEXT NOT NULL, ts REAL NOT NULL,
  PRIMARY KEY (execution, artifact, type));
CREATE TABLE IF NOT EXISTS associations (
  context INTEGER NOT NULL, execution INTEGER NOT NULL, PRIMARY KEY (context, execution));
CREATE TABLE IF NOT EXISTS attributions (
  context INTEGER NOT NULL, artifact INTEGER NOT NULL, PRIMARY KEY (context, artifact));
"""

STATES = ("NEW", "RUNNING", "COMPLETE", "FAILED", "CACHED", "CANCELED")


def db_path() -> str:
    from .runtime.storage import mxtrain_home
    return os.path.join(mxtrain_home(), "pipelines", "metadata.db")


def _connect(path: Optional[str] = None) -> sqlite3.Connection:
    path = path or db_path()
    os.makedirs(os.path.dirname(path), exist_ok=True)
    con = sqlite3.connect(path, timeout=30)
    con.execute("PRAGMA journal_mode=WAL")
    con.executescript(_SCHEMA)
    return con


@contextmanager
def _tx(path: str):
    """One transaction on a fresh connection, committed (or rolled back) and closed."""
    con = _connect(path)
    try:
        with con:
            yield con
    finally:
        con.close()


def _js(d: Optional[Dict]) -> str:
    return json.dumps(d or {}, sort_keys=True, default=str)


def digest_of(obj) -> str:
    return hashlib.sha256(json.dumps(obj, sort_keys=True, default=str).encode()).hexdigest()[:32]


class Store:
    """The metadata store (one SQLite file; safe across the API server's run threads and
    concurrent processes through SQLite's own locking)."""

    def __init__(self, path: Optional[str] = None):
        self.path = path or db_path()

    # ----------------------------------------------------------------------- writes
    def put_context(self, type_: str, name: str, properties: Optional[Dict] = None,
                    parent: Optional[int] = None) -> int:
        with _LOCK, _tx(self.path) as con:
            con.execute("INSERT OR IGNORE INTO contexts (type, name, properties, created) VALUES (?, ?, ?, ?)",
                        (type_, name, _js(properties), time.time()))
            if properties:
                con.execute("UPDATE contexts SET properties = ? WHERE type = ? AND name = ?",
                            (_js(properties), type_, name))
            cid = con.execute("SELECT id FROM contexts WHERE type = ? AND name = ?", (type_, name)).fetchone()[0]
            if parent is not None:
                con.execute("INSERT OR IGNORE INTO parent_contexts (child, parent) VALUES (?, ?)", (cid, parent))
            return cid

    def put_execution(self, type_: str, name: str, properties: Optional[Dict] = None, state: str = "NEW",
                      contexts: Optional[List[int]] = None) -> int:
        assert state in STATES, state
        now = time.time()
        with _LOCK, _tx(self.path) as con:
            eid = con.execute("INSERT INTO executions (type, name, state, properties, created, updated) "
                              "VALUES (?, ?, ?, ?, ?, ?)", (type_, name, state, _js(properties), now, now)).lastrowid
            for c in contexts or []:
                con.execute("INSERT OR IGNORE INTO associations (context, execution) VALUES (?, ?)", (c, eid))
            return eid

    def update_execution(self, eid: int, state: Optional[str] = None, properties: Optional[Dict] = None) -> None:
        with _LOCK, _tx(self.path) as con:
            row = con.execute("SELECT state, properties FROM executions WHERE id = ?", (eid,)).fetchone()
            if row is None:
                raise KeyError(f"execution {eid}")
            props = json.loads(row[1])
            props.update(properties or {})
            if state is not None:
                assert state in STATES, state
            con.execute("UPDATE executions SET state = ?, properties = ?, updated = ? WHERE id = ?",
                        (state or row[0], _js(props), time.time(), eid))

    def put_artifact(self, type_: str, uri: str, digest: str = "", properties: Optional[Dict] = None,
                     contexts: Optional[List[int]] = None) -> int:
        """An artifact is identified by (type, uri, digest): the same input read by many
        executions is one artifact."""
        with _LOCK, _tx(self.path) as con:
            con.execute("INSERT OR IGNORE INTO artifacts (type, uri, digest, properties, created) "
                        "VALUES (?, ?, ?, ?, ?)", (type_, uri, digest, _js(properties), time.time()))
            aid = con.execute("SELECT id FROM artifacts WHERE type = ? AND uri = ? AND digest = ?",
                              (type_, uri, digest)).fetchone()[0]
            for c in contexts or []:
                con.execute("INSERT OR IGNORE INTO attributions (context, artifact) VALUES (?, ?)", (c, aid))
            return aid

    def put_event(self, execution: int, artifact: int, type_: str) -> None:
        assert type_ in ("INPUT", "OUTPUT"), type_
        with _LOCK, _tx(self.path) as con:
            con.execute("INSERT OR IGNORE INTO events (execution, artifact, type, ts) VALUES (?, ?, ?, ?)",
                        (execution, artifact, type_, time.time()))

    # ------------------------------------------------------------------------ reads
    def _rows(self, sql: str, args=()) -> List[sqlite3.Row]:
        con = _connect(self.path)
        con.row_factory = sqlite3.Row
        try:
            return con.execute(sql, args).fetchall()
        finally:
            con.close()

    @staticmethod
    def _execution(r) -> Dict:
        return {"id": r["id"], "type": r["type"], "name": r["name"], "state": r["state"],
                "properties": json.loads(r["properties"]), "created": r["created"], "updated": r["updated"]}

    @staticmethod
    def _artifact(r) -> Dict:
        return {"id": r["id"], "type": r["type"], "uri": r["uri"], "digest": r["digest"],
                "properties": json.loads(r["properties"]), "created": r["created"]}

    def context(self, type_: str, name: str) -> Optional[Dict]:
        rows = self._rows("SELECT * FROM contexts WHERE type = ? AND name = ?", (type_, name))
        if not rows:
            return None
        r = rows[0]
        parents = self._rows("SELECT c.type, c.name FROM parent_contexts p JOIN contexts c ON c.id = p.parent "
                             "WHERE p.child = ?", (r["id"],))
        return {"id": r["id"], "type": r["type"], "name": r["name"], "properties": json.loads(r["properties"]),
                "created": r["created"], "parents": [{"type": p["type"], "name": p["name"]} for p in parents]}

    def executions_of(self, context_id: int) -> List[Dict]:
        return [self._execution(r) for r in self._rows(
            "SELECT e.* FROM executions e JOIN associations a ON a.execution = e.id WHERE a.context = ? "
            "ORDER BY e.id", (context_id,))]

    def execution(self, eid: int) -> Dict:
        rows = self._rows("SELECT * FROM executions WHERE id = ?", (eid,))
        if not rows:
            raise KeyError(f"execution {eid}")
        return self._execution(rows[0])

    def artifact(self, aid: int) -> Dict:
        rows = self._rows("SELECT * FROM artifacts WHERE id = ?", (aid,))
        if not rows:
            raise KeyError(f"artifact {aid}")
        return self._artifact(rows[0])

    def events_of_execution(self, eid: int) -> Dict[str, List[Dict]]:
        out = {"INPUT": [], "OUTPUT": []}
        for r in self._rows("SELECT a.*, ev.type AS etype FROM events ev JOIN artifacts a ON a.id = ev.artifact "
                            "WHERE ev.execution = ? ORDER BY a.id", (eid,)):
            out[r["etype"]].append(self._artifact(r))
        return out

    def events_of_artifact(self, aid: int) -> Dict[str, List[int]]:
        out = {"INPUT": [], "OUTPUT": []}
        for r in self._rows("SELECT execution, type FROM events WHERE artifact = ? ORDER BY execution", (aid,)):
            out[r["type"]].append(r["execution"])
        return out

    def find_execution(self, type_: str, key: str, value) -> Optional[Dict]:
        """The newest execution of ``type_`` whose property ``key`` equals ``value``."""
        for r in self._rows("SELECT * FROM executions WHERE type = ? ORDER BY id DESC", (type_,)):
            if json.loads(r["properties"]).get(key) == value:
                return self._execution(r)
        return None


# ------------------------------------------------------------------------- lineage queries
def run_lineage(run: str, store: Optional[Store] = None) -> Dict:
    """The run context, its pipeline, and every step execution with its input and output
    artifacts (the KFP run page's lineage view)."""
    st = store or Store()
    ctx = st.context("run", run)
    if ctx is None:
        raise FileNotFoundError(f"no metadata for run {run}")
    steps = []
    for e in st.executions_of(ctx["id"]):
        ev = st.events_of_execution(e["id"])
        steps.append(dict(e, inputs=ev["INPUT"], outputs=ev["OUTPUT"]))
    return {"run": ctx, "executions": steps}


def artifact_lineage(aid: int, store: Optional[Store] = None, depth: int = 8) -> Dict:
    """Who produced an artifact (OUTPUT events) and who read it (INPUT events), walking the
    producers' inputs upstream up to ``depth`` levels."""
    st = store or Store()
    art = st.artifact(aid)
    ev = st.events_of_artifact(aid)
    upstream = []
    seen = {aid}
    frontier = list(ev["OUTPUT"])
    for _ in range(depth):
        nxt = []
        for eid in frontier:
            ex = st.execution(eid)
            ins = st.events_of_execution(eid)["INPUT"]
            upstream.append(dict(ex, inputs=[a["id"] for a in ins]))
            for a in ins:
                if a["id"] not in seen:
                    seen.add(a["id"])
                    nxt.extend(st.events_of_artifact(a["id"])["OUTPUT"])
        frontier = nxt
        if not frontier:
            break
    return {"artifact": art, "produced_by": ev["OUTPUT"], "consumed_by": ev["INPUT"], "upstream": upstream}


# --------------------------------------------------------------- pipeline-runner hooks
class RunRecorder:
    """What ``pipeline.run_pipeline`` records: contexts at run start, one execution per
    step with its input artifacts, the state transitions, the output artifact.  Metadata
    failures never fail a run (the KFP metadata writer is best-effort too): every hook
    swallows and reports its exception once."""

    def __init__(self, run: str, pipeline: Optional[str], log=print, store: Optional[Store] = None):
        self.store = store or Store()
        self.log = log
        self.ok = True
        self.ctx: List[int] = []
        try:
            pctx = self.store.put_context("pipeline", pipeline) if pipeline else None
            rctx = self.store.put_context("run", run, {"pipeline": pipeline}, parent=pctx)
            self.ctx = [c for c in (pctx, rctx) if c is not None]
        except Exception as e:  # noqa: BLE001
            self._fail(e)

    def _fail(self, e: Exception) -> None:
        if self.ok:
            self.log(f"metadata store: {type(e).__name__}: {e} (run continues without lineage)")
        self.ok = False

    def step_started(self, cfg: Dict, chart_dir: Optional[str], cache_key: Optional[str]) -> Optional[int]:
        if not self.ok:
            return None
        try:
            props = {"release": cfg.get("release_name"), "namespace": cfg.get("namespace", "default"),
                     "chart": cfg.get("chart") or cfg.get("path"), "cache_key": cache_key}
            eid = self.store.put_execution("chart_step", cfg.get("release_name") or "step", props, "RUNNING",
                                           self.ctx)
            if chart_dir:
                a = self.store.put_artifact("Chart", chart_dir, digest=_chart_digest(chart_dir),
                                            properties={"chart": props["chart"]}, contexts=self.ctx)
                self.store.put_event(eid, a, "INPUT")
            vals = cfg.get("values") or {}
            a = self.store.put_artifact("ChartValues", f"values:{cfg.get('release_name')}", digest=digest_of(vals),
                                        properties={"values": vals}, contexts=self.ctx)
            self.store.put_event(eid, a, "INPUT")
            return eid
        except Exception as e:  # noqa: BLE001
            self._fail(e)
            return None

    def step_finished(self, eid: Optional[int], cfg: Dict, rc: int, seconds: float, cached_from: Optional[str] = None,
                      cache_key: Optional[str] = None, canceled: bool = False) -> None:
        if not self.ok or eid is None:
            return
        try:
            props = {"exit_code": rc, "seconds": seconds}
            if cached_from is not None:
                # the producing execution: the newest COMPLETE one with this cache key
                src = None
                for e in reversed(self._executions_with_key(cache_key) if cache_key else []):
                    if e["id"] != eid and e["state"] == "COMPLETE":
                        src = e
                        break
                props.update(cached_from_run=cached_from, cached_from_execution=src["id"] if src else None)
                state = "CACHED"
                if src is not None:   # a cached step "outputs" what its source execution produced
                    for a in self.store.events_of_execution(src["id"])["OUTPUT"]:
                        self.store.put_event(eid, a["id"], "OUTPUT")
            else:
                state = "CANCELED" if canceled else ("COMPLETE" if rc == 0 else "FAILED")
                from .launch import release as rel
                rdir = rel.release_dir(cfg.get("release_name"), cfg.get("namespace", "default"))
                a = self.store.put_artifact("ReleaseRecord", rdir, digest=f"execution-{eid}",
                                            properties={"exit_code": rc}, contexts=self.ctx)
                self.store.put_event(eid, a, "OUTPUT")
            self.store.update_execution(eid, state, props)
        except Exception as e:  # noqa: BLE001
            self._fail(e)

    def _executions_with_key(self, key: str) -> List[Dict]:
        rows = self.store._rows("SELECT * FROM executions WHERE type = 'chart_step' ORDER BY id")
        return [Store._execution(r) for r in rows if json.loads(r["properties"]).get("cache_key") == key]


def _chart_digest(chart_dir: str) -> str:
    from .pipeline import _chart_digest as d
    return d(chart_dir)[:32]
