"""Generate tests/golden/reference_cases.json.

Every case below is a transcription (as data: inputs and expected outputs) of a
test, fixture or documented expected output held by the reference repository.
The reference is Go and cannot be run here (no Go toolchain), so
the expectations are the assertions written in the reference's own tests, cited
file:line per case.  Cases whose expectations are derived by hand from the
reference's rules rather than asserted by a reference test say so in `source`.

Run:  python tests/golden/make_golden.py   (rewrites reference_cases.json)
"""
import json
import os


def sid(i):
    return {"subject_id": i}


def sset(ns, obj, rel):
    return {"subject_set": {"namespace": ns, "object": obj, "relation": rel}}


def tup(ns, obj, rel, subj):
    d = {"namespace": ns, "object": obj, "relation": rel}
    d.update(subj)
    return d


def chk(ns, obj, rel, subj, expected, source):
    d = {"namespace": ns, "object": obj, "relation": rel, "expected": expected, "source": source}
    d.update(subj)
    return d


def leaf(subj):
    d = {"type": "leaf"}
    d.update(subj)
    return d


def union(subj, children):
    d = {"type": "union", "children": children}
    d.update(subj)
    return d


def exp(subj, depth, expected, source, error=None):
    d = {"max_depth": depth, "expected": expected, "expected_error": error, "source": source}
    d.update(subj)
    return d


CE = "internal/check/engine_test.go"
EE = "internal/expand/engine_test.go"

cases = []


def case(name, source, namespaces, tuples, checks=(), expands=(), page_size=100):
    cases.append({
        "name": name,
        "source": source,
        "namespaces": [{"name": n, "id": i} for n, i in namespaces],
        "page_size": page_size,
        "tuples": list(tuples),
        "checks": list(checks),
        "expands": list(expands),
    })


# ---------------------------------------------------------------- check engine
case("check/direct inclusion", CE + ":30-48", [("test", 1)],
     [tup("test", "object", "access", sid("user"))],
     [chk("test", "object", "access", sid("user"), True, CE + ":45-47")])

sofa = "under the sofa"
case("check/indirect inclusion level 1", CE + ":50-89", [(sofa, 1)],
     [tup(sofa, "dust", "have to remove", sset(sofa, "dust", "producer")),
      tup(sofa, "dust", "producer", sid("Mark"))],
     [chk(sofa, "dust", "have to remove", sid("Mark"), True, CE + ":80-88")])

case("check/direct exclusion", CE + ":91-117", [("object-namespace", 10)],
     [tup("object-namespace", "object-id", "relation", sid("user-id"))],
     [chk("object-namespace", "object-id", "relation", sid("not user-id"), False, CE + ":108-116")])

case("check/wrong object ID", CE + ":119-149", [("", 1)],
     [tup("", "object", "access", sset("", "object", "owner")),
      tup("", "not object", "owner", sid("user"))],
     [chk("", "object", "access", sid("user"), False, CE + ":141-148")])

diary, entry = "diary", "entry for 6. Nov 2020"
case("check/wrong relation name", CE + ":151-187", [(diary, 1)],
     [tup(diary, entry, "read", sset(diary, entry, "author")),
      tup(diary, entry, "not author", sid("your mother"))],
     [chk(diary, entry, "read", sid("your mother"), False, CE + ":178-186")])

sn, on = "some namespace", "all organizations"
case("check/indirect inclusion level 2", CE + ":189-255", [(sn, 1), (on, 2)],
     [tup(sn, "some object", "write", sset(sn, "some object", "owner")),
      tup(sn, "some object", "owner", sset(on, "some organization", "member")),
      tup(on, "some organization", "member", sid("some user"))],
     [chk(sn, "some object", "write", sid("some user"), True, CE + ":235-243"),
      chk(on, "some organization", "member", sid("some user"), True, CE + ":245-254")])

case("check/rejects transitive relation", CE + ":257-295", [("", 2)],
     [tup("", "file", "parent", sset("", "directory", "")),
      tup("", "directory", "access", sid("user"))],
     [chk("", "file", "access", sid("user"), False, CE + ":287-294")])

case("check/subject id next to subject set", CE + ":297-348", [("namesp", 1)],
     [tup("namesp", "obj", "owner", sid("u1")),
      tup("namesp", "obj", "owner", sset("namesp", "org", "member")),
      tup("namesp", "org", "member", sid("u2"))],
     [chk("namesp", "obj", "owner", sid("u1"), True, CE + ":329-337"),
      chk("namesp", "obj", "owner", sid("u2"), True, CE + ":339-347")])

case("check/paginates", CE + ":350-394", [("namesp", 1)],
     [tup("namesp", "obj", "access", sid(u)) for u in ["u1", "u2", "u3", "u4"]],
     [chk("namesp", "obj", "access", sid(u), True, CE + ":370-380") for u in ["u1", "u2", "u3", "u4"]],
     page_size=2)

wide = [tup("namesp", "obj", "access", sset("namesp", o, "member")) for o in ["o1", "o2"]]
wide += [tup("namesp", ["o1", "o2"][i % 2], "member", sid(u)) for i, u in enumerate(["u1", "u2", "u3", "u4"])]
case("check/wide tuple graph", CE + ":396-436", [("namesp", 1)], wide,
     [chk("namesp", "obj", "access", sid(u), True, CE + ":425-435") for u in ["u1", "u2", "u3", "u4"]])

mt = "munich transport"
st, od, cs = "Sendlinger Tor", "Odeonsplatz", "Central Station"
cyc = [tup(mt, st, "connected", sset(mt, od, "connected")),
       tup(mt, od, "connected", sset(mt, cs, "connected")),
       tup(mt, cs, "connected", sset(mt, st, "connected"))]
case("check/circular tuples", CE + ":438-489", [(mt, 0)], cyc,
     [chk(mt, st, "connected", sid(cs), False, CE + ":477-488")])

# --------------------------------------------------------------- check handler
CH = "internal/check/handler_test.go"
case("check/handler", CH + ":41-109", [("check handler", 0)],
     [tup("check handler", "o", "r", sid("s"))],
     [chk("not check handler", "", "", sid("foo"), False, CH + ":73-81 (unknown namespace -> denied)"),
      chk("check handler", "o", "r", sid("s"), True, CH + ":83-98"),
      chk("check handler", "", "", sid("foo"), False, CH + ":100-108 (wildcard object/relation)")])

# ----------------------------------------------------------------- CLI / docs
case("check/cli denied", "cmd/check/root_test.go:12-19", [("TestCheckCommand", 0)], [],
     [chk("TestCheckCommand", "object", "access", sid("subject"), False, "cmd/check/root_test.go:17-18")])

DOC = "contrib/docs-code-samples/simple-access-check-guide"
case("docs/simple access check", DOC, [("messages", 1)],
     [tup("messages", "02y_15_4w350m3", "decypher", sid("john"))],
     [chk("messages", "02y_15_4w350m3", "decypher", sid("john"), True,
          DOC + "/01-check-direct-access/expected_output.txt ('Allowed')")])

# --------------------------------------------------------------- expand engine
case("expand/returns SubjectID", EE + ":32-42", [], [],
     expands=[exp(sid("user"), 100, leaf(sid("user")), EE + ":36-41")])

case("expand/expands one level", EE + ":44-84", [("", 0)],
     [tup("", "boulder group", "member", sid("Tommy")),
      tup("", "boulder group", "member", sid("Paul"))],
     expands=[exp(sset("", "boulder group", "member"), 100,
                  union(sset("", "boulder group", "member"), [leaf(sid("Paul")), leaf(sid("Tommy"))]),
                  EE + ":70-83 (order pinned: Paul before Tommy)")])

two = []
for g, users in [("x", ["a", "b", "c"]), ("y", ["d", "e", "f"])]:
    two.append(tup("", "z", "transitive member", sset("", g, "member")))
    two += [tup("", g, "member", sid(u)) for u in users]
case("expand/expands two levels", EE + ":86-163", [("", 0)], two,
     expands=[exp(sset("", "z", "transitive member"), 100,
                  union(sset("", "z", "transitive member"), [
                      union(sset("", "x", "member"), [leaf(sid(u)) for u in "abc"]),
                      union(sset("", "y", "member"), [leaf(sid(u)) for u in "def"])]),
                  EE + ":160-162")])

chain = []
prev = "root"
for s in ["0", "1", "2", "3"]:
    chain.append(tup("", prev, "child", sset("", s, "child")))
    prev = s
case("expand/respects max depth", EE + ":165-221", [("", 0)], chain,
     expands=[exp(sset("", "root", "child"), 4,
                  union(sset("", "root", "child"), [
                      union(sset("", "0", "child"), [
                          union(sset("", "1", "child"), [leaf(sset("", "2", "child"))])])]),
                  EE + ":217-220")])

case("expand/paginates", EE + ":223-252", [("", 0)],
     [tup("", "root", "access", sid(u)) for u in ["u1", "u2", "u3", "u4"]],
     expands=[exp(sset("", "root", "access"), 10,
                  union(sset("", "root", "access"), [leaf(sid(u)) for u in ["u1", "u2", "u3", "u4"]]),
                  EE + ":244-250")],
     page_size=2)

case("expand/handles subject sets as leaf", EE + ":254-283", [("", 0)],
     [tup("", "root", "rel", sset("", "so", "sr"))],
     expands=[exp(sset("", "root", "rel"), 100,
                  union(sset("", "root", "rel"), [leaf(sset("", "so", "sr"))]), EE + ":279-282")])

case("expand/circular tuples", EE + ":285-356", [(mt, 0)], cyc,
     expands=[exp(sset(mt, st, "connected"), 100,
                  union(sset(mt, st, "connected"), [
                      union(sset(mt, od, "connected"), [
                          union(sset(mt, cs, "connected"), [leaf(sset(mt, st, "connected"))])])]),
                  EE + ":347-355")])

EH = "internal/expand/handler_test.go"
case("expand/handler", EH + ":24-108", [("expand handler", 0)],
     [tup("expand handler", "root", "parent of", sid("child0")),
      tup("expand handler", "root", "parent of", sid("child1"))],
     expands=[exp(sset("not expand handler", "", ""), 10, None, EH + ":48-59 (404 Unknown namespace)",
                  error="not_found"),
              exp(sset("expand handler", "root", "parent of"), 2,
                  union(sset("expand handler", "root", "parent of"), [leaf(sid("child0")), leaf(sid("child1"))]),
                  EH + ":61-107")])

case("expand/cli unknown tuple", "cmd/expand/root_test.go:14-31", [("TestExpandCommand", 0)], [],
     expands=[exp(sset("TestExpandCommand", "object", "access"), 100, None,
                  "cmd/expand/root_test.go:20-23 ('null')")])

DOCX = "contrib/docs-code-samples/expand-api-display-access"
beach = [
    tup("directories", "/photos", "owner", sid("maureen")),
    tup("files", "/photos/beach.jpg", "owner", sid("maureen")),
    tup("files", "/photos/mountains.jpg", "owner", sid("laura")),
    tup("directories", "/photos", "access", sid("laura")),
    tup("directories", "/photos", "access", sset("directories", "/photos", "owner")),
    tup("files", "/photos/beach.jpg", "access", sset("files", "/photos/beach.jpg", "owner")),
    tup("files", "/photos/beach.jpg", "access", sset("directories", "/photos", "access")),
    tup("files", "/photos/mountains.jpg", "access", sset("files", "/photos/mountains.jpg", "owner")),
    tup("files", "/photos/mountains.jpg", "access", sset("directories", "/photos", "access")),
]
here = os.path.dirname(os.path.abspath(__file__))
# expected_output.txt of 01-expand-beach, transcribed as data (SQLite order: subject
# sets before subject IDs, namespace id 1 before 2).
beach_tree = union(sset("files", "/photos/beach.jpg", "access"), [
    union(sset("files", "/photos/beach.jpg", "owner"), [leaf(sid("maureen"))]),
    union(sset("directories", "/photos", "access"), [
        leaf(sset("directories", "/photos", "owner")),
        leaf(sid("laura"))])])
case("docs/expand beach", DOCX + "/00-create-tuples/cli.sh", [("files", 1), ("directories", 2)], beach,
     checks=[chk("files", "/photos/beach.jpg", "access", sid("laura"), True,
                 "docs/docs/guides/expand-api-display-who-has-access.mdx (laura has access via /photos); hand-derived"),
             chk("files", "/photos/mountains.jpg", "access", sid("maureen"), True,
                 "hand-derived from the same tuples (maureen owns /photos)")],
     expands=[exp(sset("files", "/photos/beach.jpg", "access"), 3, beach_tree,
                  DOCX + "/01-expand-beach/expected_output.txt")])

# -------------------------------------------------------- cat videos (config #1)
CV = "contrib/cat-videos-example/relation-tuples/*.json"
cat = [
    tup("videos", "/cats/1.mp4", "owner", sset("videos", "/cats", "owner")),
    tup("videos", "/cats/1.mp4", "view", sset("videos", "/cats/1.mp4", "owner")),
    tup("videos", "/cats/1.mp4", "view", sid("*")),
    tup("videos", "/cats/2.mp4", "owner", sset("videos", "/cats", "owner")),
    tup("videos", "/cats/2.mp4", "view", sset("videos", "/cats/2.mp4", "owner")),
    tup("videos", "/cats", "owner", sid("cat lady")),
    tup("videos", "/cats", "view", sset("videos", "/cats", "owner")),
]
HD = "hand-derived (SURVEY.md 8(c) config #1)"
v = lambda o, r: sset("videos", o, r)
case("config1/cat videos", CV + " + contrib/cat-videos-example/keto.yml", [("videos", 0)], cat,
     checks=[chk("videos", "/cats/1.mp4", "view", sid("*"), True, HD),
             chk("videos", "/cats/1.mp4", "view", sid("cat lady"), True, HD),
             chk("videos", "/cats/2.mp4", "view", sid("cat lady"), True, HD),
             chk("videos", "/cats", "owner", sid("cat lady"), True, HD),
             chk("videos", "/cats", "view", sid("cat lady"), True, HD),
             chk("videos", "/cats/2.mp4", "view", sid("*"), False, HD),
             chk("videos", "/cats/1.mp4", "owner", sid("*"), False, HD)],
     expands=[exp(v("/cats/2.mp4", "view"), 100,
                  union(v("/cats/2.mp4", "view"), [union(v("/cats/2.mp4", "owner"), [
                      union(v("/cats", "owner"), [leaf(sid("cat lady"))])])]), HD),
              exp(v("/cats/2.mp4", "view"), 2,
                  union(v("/cats/2.mp4", "view"), [leaf(v("/cats/2.mp4", "owner"))]), HD),
              exp(v("/cats/2.mp4", "view"), 1, leaf(v("/cats/2.mp4", "view")), HD),
              exp(v("/cats/2.mp4", "view"), 0, None, HD),
              exp(v("/cats/1.mp4", "view"), 100,
                  union(v("/cats/1.mp4", "view"), [
                      union(v("/cats/1.mp4", "owner"), [union(v("/cats", "owner"), [leaf(sid("cat lady"))])]),
                      leaf(sid("*"))]), HD + " (SQLite NULL-first order)")])

if __name__ == "__main__":
    out = os.path.join(here, "reference_cases.json")
    with open(out, "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "cases": cases}, f, indent=1, sort_keys=False)
        f.write("\n")
    n_chk = sum(len(c["checks"]) for c in cases)
    n_exp = sum(len(c["expands"]) for c in cases)
    print(f"wrote {out}: {len(cases)} cases, {n_chk} checks, {n_exp} expands")
