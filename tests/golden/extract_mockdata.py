"""Extract the reference's own test fixtures (data only) into JSON.

Run once in the survey/build container, where /root/reference exists:

    python tests/golden/extract_mockdata.py

The reference keeps its fixtures as TypeScript object literals in
``tests/MockData.ts`` / ``tests/MockData2.ts``.  This script cuts each named
literal out of the file, drops the ``: Type[]`` annotation of its ``const``
line, and lets the local Node (v12) evaluate the literal with the few free
identifiers it references bound to fixed stand-ins (``Yesterday``/``Today`` are
pinned to constants, and so is ``Date.now``, so the output is deterministic).  Only the resulting JSON
*data* is committed under ``tests/fixtures/``; no reference source is kept.
Properties whose value is ``undefined`` are dropped, exactly as Jest's
``toEqual`` ignores them.
"""
import json
import os
import re
import subprocess
import sys

REF = "/root/reference/tests"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fixtures")

# fixed stand-ins for the time-dependent constants (MockData.ts:3951-3952)
TODAY = 1700000000000
YESTERDAY = TODAY - 86400000

PRELUDE = f"""
Date.now = () => {TODAY};
const Today = {TODAY};
const Yesterday = {YESTERDAY};
const Service = "srv";
const Namespace = "ns";
const Version = "latest";
const UniqueServiceName = `${{Service}}\\t${{Namespace}}\\t${{Version}}`;
const UniqueEndpointName = `${{UniqueServiceName}}\\tGET\\thttp://srv/api/a`;
const Method = "GET";
const Status = "200";
const Utils = {{ ObjectToInterfaceString: (o) => "__schema__" + JSON.stringify(o),
                BelongsToMinuteTimestamp: (t) => t - (t % 60000) }};
"""

WANT = {
    "MockData.ts": [
        "MockTrace",
        "MockEndpointDependencies",
        "MockTracePDAS",
        "MockRlDataPDAS",
        "MockEndpointDependenciesPDAS",
        "MockBaseRlData1",
        "MockBaseCrlData1",
        "MockBaseCrlData2",
        "MockCombinedBaseData",
        "MockReplicas",
        "MockDependencies",
        "MockEndpointInfoPDAS1",
        "MockHistoricalData",
    ],
    "MockData2.ts": ["traces"],
}


def cut_literal(text, name):
    m = re.search(r"^const %s(\s*:\s*[A-Za-z_\[\]]+)?\s*=\s*" % re.escape(name), text, re.M)
    if not m:
        raise KeyError(name)
    i = m.end()
    open_ch = text[i]
    close_ch = {"[": "]", "{": "}"}[open_ch]
    depth, j, in_str, quote = 0, i, False, ""
    while True:
        c = text[j]
        if in_str:
            if c == "\\":
                j += 2
                continue
            if c == quote:
                in_str = False
        elif c in "\"'`":
            in_str, quote = True, c
        elif c == open_ch:
            depth += 1
        elif c == close_ch:
            depth -= 1
            if depth == 0:
                return text[i : j + 1]
        j += 1


def cut_expression(text, name):
    """`const NAME = <expression>;` for a non-literal expression (MockLogsPDAS
    is a template string split into lines, MockData.ts:3933-3941)."""
    m = re.search(r"^const %s\s*=\s*" % re.escape(name), text, re.M)
    if not m:
        raise KeyError(name)
    i = m.end()
    j, in_str, quote, depth = i, False, "", 0
    while True:
        c = text[j]
        if in_str:
            if c == "\\":
                j += 2
                continue
            if c == quote:
                in_str = False
        elif c in "\"'`":
            in_str, quote = True, c
        elif c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        elif c == ";" and depth == 0:
            return text[i:j]
        j += 1


EXPRESSIONS = {"MockData.ts": ["MockLogsPDAS"]}


def main():
    os.makedirs(OUT, exist_ok=True)
    for fname, names in EXPRESSIONS.items():
        text = open(os.path.join(REF, fname)).read()
        for name in names:
            js = "const __v = " + cut_expression(text, name) + ";\nprocess.stdout.write(JSON.stringify(__v));\n"
            out = subprocess.run(["node", "-e", js], check=True, capture_output=True, text=True).stdout
            dst = os.path.join(OUT, f"{name}.json")
            with open(dst, "w") as f:
                json.dump(json.loads(out), f, indent=1, ensure_ascii=False)
            print("wrote", dst, file=sys.stderr)
    for fname, names in WANT.items():
        text = open(os.path.join(REF, fname)).read()
        # MockBaseCrlData2 needs divBaseData2 (MockData.ts:4501-4504)
        extra = ""
        if fname == "MockData.ts":
            m = re.search(r"^const divBaseData2 = ([\s\S]*?);\n", text, re.M)
            extra = "const divBaseData2 = " + m.group(1) + ";\n"
        for name in names:
            lit = cut_literal(text, name)
            js = PRELUDE + extra + "const __v = " + lit + ";\nprocess.stdout.write(JSON.stringify(__v));\n"
            out = subprocess.run(["node", "-e", js], check=True, capture_output=True, text=True).stdout
            data = json.loads(out)
            dst = os.path.join(OUT, f"{name}.json" if fname == "MockData.ts" else "MockData2_traces.json")
            with open(dst, "w") as f:
                json.dump(data, f, indent=1, sort_keys=False)
            print("wrote", dst, file=sys.stderr)


if __name__ == "__main__":
    main()
