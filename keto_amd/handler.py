"""Check / expand request handling over the MI355X engines, and the batch-check endpoint.

Mirrors the reference's REST handlers (status mapping and request parsing), which stay
unchanged in a Go deployment — here they are the harness that shows a
caller gets the reference's responses from the new engines:

    GET  /check    internal/check/handler.go:85-107   200 {"allowed":true} | 403 {"allowed":false} | 400
    POST /check    internal/check/handler.go:128-146  same; a JSON decode error is 400
    GET  /expand   internal/expand/handler.go:78-92   200 tree | null, 400 bad max-depth, 404 unknown namespace
    POST /check/batch  (new)    200 {"results": [{"allowed": bool} | {"error": ...}]}

URL parsing restates RelationQuery.FromURLQuery (internal/relationtuple/definitions.go:
458-493): a bare "subject" key, both subject forms, or an incomplete subject_set are 400;
missing namespace/object/relation are "" (no filter, R5).  Deliberate divergence: the
reference's postCheck writes its 400 for a bad body and then goes on to evaluate a zero
tuple (handler.go:130-132); here the 400 is the whole response.

The batch endpoint takes many tuples in one request and answers them through the engine's
throughput path (check.Engine.check_batch: ketogpu_resolve_batch, then ONE
ketogpu_check_ids — chunked H2D overlapped with the traversal, one D2H — with only
wildcard-root and R4-flagged requests re-answered sequentially), per-tuple errors inline.
`python -m keto_amd.handler --port P --tuples FILE --namespaces a:1,b:2` serves these
routes with http.server (a demo harness; the production server is Keto's own).
"""
import json
from urllib.parse import parse_qs

from . import check, expand
from .relationtuple import InternalRelationTuple, NilSubject, SubjectID, SubjectSet

SUBJECT_ID = "subject_id"
SS_KEYS = ("subject_set.namespace", "subject_set.object", "subject_set.relation")


class BadRequest(ValueError):
    """herodot.ErrBadRequest (HTTP 400)"""


def _get(q, k):
    v = q.get(k)
    if v is None:
        return None
    return v[0] if isinstance(v, (list, tuple)) else v


def relation_query_from_url(q):
    """RelationQuery.FromURLQuery (definitions.go:458-493) -> (namespace, object, relation, subject|None)"""
    if "subject" in q:
        raise BadRequest('provide "subject_id" or "subject_set.*"; support for "subject" was dropped')
    has_id = SUBJECT_ID in q
    has_ss = [k in q for k in SS_KEYS]
    subject = None
    if not has_id and not any(has_ss):
        pass
    elif has_id and all(has_ss):
        raise BadRequest("exactly one of subject_set or subject_id has to be provided")
    elif has_id:
        subject = SubjectID(_get(q, SUBJECT_ID))
    elif all(has_ss):
        subject = SubjectSet(*(_get(q, k) for k in SS_KEYS))
    else:
        raise BadRequest('incomplete subject, provide "subject_id" or a complete "subject_set.*"')
    return _get(q, "namespace") or "", _get(q, "object") or "", _get(q, "relation") or "", subject


def tuple_from_url(q):
    """InternalRelationTuple.FromURLQuery (definitions.go:378-395): the subject is required"""
    ns, obj, rel, subject = relation_query_from_url(q)
    if subject is None:
        raise BadRequest("Subject has to be specified.")
    return InternalRelationTuple(ns, obj, rel, subject)


def _json_string(d, k):
    """a string field of the JSON tuple: Go's decoder turns null into "" and rejects any
    other non-string value (json.UnmarshalTypeError -> 400)"""
    v = d.get(k)
    if v is None:
        return ""
    if not isinstance(v, str):
        raise BadRequest(f"json: cannot unmarshal {type(v).__name__} into field {k} of type string")
    return v


def tuple_from_json(d):
    """JSON body of POST /check: {namespace, object, relation, subject_id | subject_set}"""
    if not isinstance(d, dict):
        raise BadRequest("Unable to decode JSON payload: expected an object")
    # the reference decodes into *string / *SubjectSet (definitions.go:316-325): a key
    # holding null is the same as an absent key
    if d.get("subject_id") is not None and d.get("subject_set") is not None:
        raise BadRequest("exactly one of subject_set or subject_id has to be provided")
    ns, obj, rel = (_json_string(d, k) for k in ("namespace", "object", "relation"))
    subject = None
    if d.get("subject_id") is not None:
        subject = SubjectID(_json_string(d, "subject_id"))
    elif d.get("subject_set") is not None:
        ss = d["subject_set"]
        if not isinstance(ss, dict):
            raise BadRequest(f"json: cannot unmarshal {type(ss).__name__} into field subject_set of type object")
        subject = SubjectSet(*(_json_string(ss, k) for k in ("namespace", "object", "relation")))
    return InternalRelationTuple(ns, obj, rel, subject)


def _underscore_ok(s):
    """Go's strconv underscoreOK: '_' only between digits or after a base prefix"""
    saw, i = "^", 0
    if s[:1] in ("-", "+"):
        s = s[1:]
    hexa = False
    if len(s) >= 2 and s[0] == "0" and s[1].lower() in "box":
        i, saw, hexa = 2, "0", s[1].lower() == "x"
    while i < len(s):
        c = s[i]
        if c.isdigit() and c.isascii() or hexa and c.lower() in "abcdef":
            saw = "0"
        elif c == "_":
            if saw != "0":
                return False
            saw = "_"
        else:
            if saw == "_":
                return False
            saw = "!"
        i += 1
    return saw != "_"


def go_parse_int(s):
    """strconv.ParseInt(s, 0, 64), as getExpand parses max-depth (internal/expand/handler.go:79):
    an optional sign, then 0b/0o/0x prefixes or a leading 0 for octal, '_' digit
    separators, no whitespace; ValueError on bad syntax or a value outside int64"""
    if not isinstance(s, str) or not s:
        raise ValueError("invalid syntax")
    neg = s[0] == "-"
    body = s[1:] if s[0] in "+-" else s
    if not body:
        raise ValueError("invalid syntax")
    base, digits = 10, body
    if body[0] == "0":
        p = body[1:2].lower()
        if len(body) >= 3 and p in ("b", "o", "x"):
            base, digits = {"b": 2, "o": 8, "x": 16}[p], body[2:]
        else:
            base, digits = 8, body[1:]
    n, underscores = 0, False
    for c in digits:
        if c == "_":
            underscores = True
            continue
        d = int(c, 16) if c.isascii() and c.lower() in "0123456789abcdef" else 99
        if d >= base:
            raise ValueError("invalid syntax")
        n = n * base + d
    if underscores and not _underscore_ok(s):
        raise ValueError("invalid syntax")
    if (not neg and n >= 1 << 63) or (neg and n > 1 << 63):
        raise ValueError("value out of range")
    return -n if neg else n


class Handler:
    """(status, JSON body) for each route; engines are check.Engine and expand.Engine"""

    def __init__(self, check_engine: check.Engine, expand_engine: expand.Engine):
        self.check = check_engine
        self.expand = expand_engine

    @staticmethod
    def _error(code, reason):
        status = {400: "Bad Request", 404: "Not Found", 500: "Internal Server Error"}[code]
        return code, {"error": {"code": code, "status": status, "reason": reason}}

    def _allowed(self, t):
        try:
            ok = self.check.SubjectIsAllowed(t)
        except NilSubject:
            return self._error(400, "Subject has to be specified.")
        return (200, {"allowed": True}) if ok else (403, {"allowed": False})

    def get_check(self, query):
        q = parse_qs(query, keep_blank_values=True) if isinstance(query, str) else query
        try:
            t = tuple_from_url(q)
        except BadRequest as e:
            return self._error(400, str(e))
        return self._allowed(t)

    def post_check(self, body):
        try:
            t = tuple_from_json(json.loads(body))
        except (ValueError, BadRequest) as e:
            return self._error(400, f"Unable to decode JSON payload: {e}")
        return self._allowed(t)

    def get_expand(self, query):
        q = parse_qs(query, keep_blank_values=True) if isinstance(query, str) else query
        raw = _get(q, "max-depth")
        try:
            depth = go_parse_int(raw)  # strconv.ParseInt(s, 0, 0)
        except ValueError as e:
            # Go's Query().Get gives "" for a missing key; strconv quotes with escapes
            return self._error(400, f"strconv.ParseInt: parsing {json.dumps(raw or '')}: {e}")
        # ketogpu_expand takes an int32: every depth beyond any tree's height acts the same
        depth = max(-1, min(depth, 2**31 - 1))
        subject = SubjectSet(_get(q, "namespace") or "", _get(q, "object") or "", _get(q, "relation") or "")
        try:
            tree = self.expand.BuildTree(subject, depth)
        except expand.NotFound as e:
            return self._error(404, str(e))
        return 200, (tree.to_node() if tree else None)

    def post_check_batch(self, body):
        """{"tuples": [...]} -> {"results": [...]}, one engine call for the whole batch"""
        try:
            d = json.loads(body)
            items = d["tuples"] if isinstance(d, dict) else d
            if not isinstance(items, list):
                raise BadRequest("expected a list of relation tuples")
        except (ValueError, KeyError, TypeError, BadRequest) as e:
            return self._error(400, f"Unable to decode JSON payload: {e}")
        results = [None] * len(items)
        tuples, where = [], []
        for i, it in enumerate(items):
            try:
                t = tuple_from_json(it)
                if t.subject is None:
                    raise BadRequest("Subject has to be specified.")
                tuples.append(t)
                where.append(i)
            except (BadRequest, ValueError, AttributeError) as e:
                results[i] = {"error": {"code": 400, "reason": str(e)}}
        batch = (getattr(self.check, "check_batch", None) or self.check.check_many) if tuples else None
        for i, ok in zip(where, batch(tuples) if tuples else []):
            results[i] = {"allowed": bool(ok)}
        return 200, {"results": results}


def serve(handler: Handler, port: int):  # pragma: no cover - demo harness
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
    from urllib.parse import urlsplit

    class H(BaseHTTPRequestHandler):
        def _send(self, code, body):
            data = json.dumps(body).encode()
            self.send_response(code)
            self.send_header("Content-Type", "application/json")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        def do_GET(self):
            u = urlsplit(self.path)
            if u.path == "/check":
                self._send(*handler.get_check(u.query))
            elif u.path == "/expand":
                self._send(*handler.get_expand(u.query))
            else:
                self._send(404, {"error": {"code": 404, "status": "Not Found"}})

        def do_POST(self):
            body = self.rfile.read(int(self.headers.get("Content-Length", 0) or 0))
            path = urlsplit(self.path).path
            if path == "/check":
                self._send(*handler.post_check(body))
            elif path == "/check/batch":
                self._send(*handler.post_check_batch(body))
            else:
                self._send(404, {"error": {"code": 404, "status": "Not Found"}})

    ThreadingHTTPServer(("127.0.0.1", port), H).serve_forever()


def main():  # pragma: no cover - demo harness
    import argparse

    from .snapshot import Snapshot
    p = argparse.ArgumentParser()
    p.add_argument("--port", type=int, default=4466)
    p.add_argument("--tuples", required=True, help="file with one relation tuple string per line")
    p.add_argument("--namespaces", required=True, help="name:id,name:id")
    a = p.parse_args()
    ns = [(x.split(":")[0], int(x.split(":")[1])) for x in a.namespaces.split(",")]
    tuples = [InternalRelationTuple.FromString(line.strip()) for line in open(a.tuples) if line.strip()]
    snap = Snapshot.from_tuples(ns, tuples)
    serve(Handler(check.Engine(snap), expand.Engine(snap)), a.port)


if __name__ == "__main__":
    main()
