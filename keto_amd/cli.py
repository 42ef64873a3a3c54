"""`keto check` mirror with a batch mode.

The reference CLI checks one tuple per call over gRPC (cmd/check/root.go:25-61:
`keto check <subject> <relation> <namespace> <object>`, output "Allowed" / "Denied", or
{"allowed": bool} with --format json).  The batch mode reads relation tuples in the
reference's human-readable form, one per line — parsed exactly as `keto relation-tuple
parse` does (cmd/relationtuple/parse.go:47-87: trimmed lines, blank lines and `//`
comments skipped, InternalRelationTuple.FromString, definitions.go:277-306) — and answers
all of them with one engine batch (check.Engine.check_batch: resolve on the host, one
host-to-host GPU call).  The network comes from a tuple file (--tuples, same format) or
a persisted snapshot (--snapshot), as the CLI here has no server to ask.

    python -m keto_amd.cli check alice view videos /cats/1.mp4 --tuples t.txt --namespaces videos:0
    python -m keto_amd.cli check --batch queries.txt --tuples t.txt --namespaces videos:0 [--format json]
"""
import argparse
import json
import sys

from .relationtuple import InternalRelationTuple, MalformedInput, SubjectID


class CliError(Exception):
    """a failure already reported on stderr (cmdx.FailSilently)"""


def parse_file(path, stdin=None, stderr=None):
    """parseFile (cmd/relationtuple/parse.go:47-87) -> list of InternalRelationTuple"""
    stderr = stderr or sys.stderr
    name = "stdin" if path == "-" else path
    try:
        text = (stdin or sys.stdin).read() if path == "-" else open(path, encoding="utf-8").read()
    except OSError as e:
        print(f"Could not open file {path}: {e}", file=stderr)
        raise CliError(path) from None
    out = []
    for i, row in enumerate(text.split("\n")):
        row = row.strip()
        if not row or row.startswith("//"):
            continue
        try:
            out.append(InternalRelationTuple.FromString(row))
        except MalformedInput as e:
            print(f"Could not decode {name}:{i + 1}\n  {row}\n\n{e}", file=stderr)
            raise CliError(name) from None
    return out


def _namespaces(spec):
    out = []
    for part in spec.split(","):
        name, _, nid = part.rpartition(":")
        out.append((name, int(nid)))
    return out


def _engine(a):
    from . import check
    from .snapshot import Snapshot
    if a.snapshot:
        snap = Snapshot.load(a.snapshot)
    else:
        snap = Snapshot.from_tuples(_namespaces(a.namespaces), parse_file(a.tuples))
    return check.Engine(snap, device=a.device)


def main(argv=None, stdout=None, stderr=None, stdin=None):
    stdout, stderr = stdout or sys.stdout, stderr or sys.stderr
    p = argparse.ArgumentParser(prog="keto")
    sub = p.add_subparsers(dest="cmd", required=True)
    c = sub.add_parser("check", help="Check whether a subject has a relation on an object")
    c.add_argument("args", nargs="*", metavar="<subject> <relation> <namespace> <object>")
    c.add_argument("--batch", help="file of relation tuples (namespace:object#relation@subject), '-' = stdin")
    c.add_argument("--tuples", help="the network: a file of relation tuples")
    c.add_argument("--snapshot", help="the network: a persisted snapshot (ketogpu_snapshot_save)")
    c.add_argument("--namespaces", default="", help="name:id,name:id (with --tuples)")
    c.add_argument("--format", choices=["default", "json"], default="default")
    c.add_argument("--device", type=int, default=0)
    a = p.parse_args(argv)
    if not ((a.batch and not a.args) or (not a.batch and len(a.args) == 4)):
        print("accepts 4 arg(s) <subject> <relation> <namespace> <object>, or --batch FILE", file=stderr)
        return 1
    if not a.tuples and not a.snapshot:
        print("the network: --tuples FILE (with --namespaces) or --snapshot FILE", file=stderr)
        return 1
    try:
        if a.batch:
            tuples = parse_file(a.batch, stdin=stdin, stderr=stderr)
        else:  # cmd/check/root.go:41-49: the subject argument is a subject id
            subject, relation, namespace, obj = a.args
            tuples = [InternalRelationTuple(namespace, obj, relation, SubjectID(subject))]
        eng = _engine(a)
    except CliError:
        return 1
    got = eng.check_batch(tuples)
    if a.format == "json":
        body = [{"allowed": bool(x)} for x in got]
        print(json.dumps(body[0] if not a.batch else {"results": body}), file=stdout)
    else:
        for x in got:
            print("Allowed" if x else "Denied", file=stdout)
    return 0


if __name__ == "__main__":
    sys.exit(main())
