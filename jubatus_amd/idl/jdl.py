"""Parser of the Jubatus IDL language (the jenerator input format).

Reference: tools/jenerator/src/{jdl_lexer.mll,jdl_parser.mly,syntax.ml}
(OCaml). Grammar handled here:

    file     := (message | exception | typedef | enum | service | comment | include)*
    include  := "%include" text                      (a C++ header hint; ignored)
    message  := "message" NAME ["(" STRING ")"] "{" (INT ":" type NAME)* "}"
    typedef  := "type" NAME "=" type
    enum     := "enum" NAME "{" (INT ":" NAME)* "}"
    service  := "service" NAME "{" method* "}"
    method   := doc* decorator* type NAME "(" [INT ":" type NAME ("," ...)*] ")"
    type     := NAME ["<" type ("," type)* ">"]
    doc      := "#-" text        decorator := "#@" WORD ["(" INT ")"]

Decorators: routing random | broadcast | cht[(n)] (default n=2) | internal;
request type update | analysis | nolock; aggregator pass | all_and | all_or |
merge | concat | add | ignore (syntax.ml:111-130).
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field

ROUTINGS = ("random", "broadcast", "cht", "internal")
LOCKS = ("update", "analysis", "nolock")
AGGS = ("pass", "all_and", "all_or", "merge", "concat", "add", "ignore")


class IdlError(ValueError):
    def __init__(self, msg: str, line: int):
        super().__init__(f"line {line}: {msg}")
        self.line = line


@dataclass
class Field:
    index: int
    type: str
    name: str


@dataclass
class Message:
    name: str
    fields: list[Field]
    native: str = ""       # the optional ("c++ type") annotation
    exception: bool = False


@dataclass
class IdlMethod:
    name: str
    ret: str
    args: list[Field]
    routing: str = "random"
    cht_n: int = 2
    lock: str = "update"
    agg: str = "pass"
    doc: list[str] = field(default_factory=list)


@dataclass
class Service:
    name: str
    methods: list[IdlMethod]


@dataclass
class IdlFile:
    messages: list[Message] = field(default_factory=list)
    typedefs: dict[str, str] = field(default_factory=dict)
    enums: dict[str, list[tuple[int, str]]] = field(default_factory=dict)
    services: list[Service] = field(default_factory=list)


_TOKEN = re.compile(r"""
    (?P<include>%include[^\n]*) |
    (?P<doc>\#-[^\n]*) |
    (?P<deco>\#@[A-Za-z_]+(?:\(\s*\d+\s*\))?) |
    (?P<comment>\#[^\n]*) |
    (?P<string>"[^"]*") |
    (?P<int>\d+) |
    (?P<name>[A-Za-z_][A-Za-z0-9_]*) |
    (?P<punct>[{}()<>:,=]) |
    (?P<nl>\n) |
    (?P<ws>[ \t\r]+) |
    (?P<bad>.)
""", re.X)


def tokenize(text: str) -> list[tuple[str, str, int]]:
    toks, line = [], 1
    for m in _TOKEN.finditer(text):
        kind = m.lastgroup
        v = m.group()
        if kind == "nl":
            line += 1
            continue
        if kind in ("ws", "comment", "include"):   # %include: C++ header hint only
            continue
        if kind == "bad":
            raise IdlError(f"unexpected character {v!r}", line)
        toks.append((kind, v, line))
    return toks


class _Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0

    def peek(self, k: int = 0):
        j = self.i + k
        return self.t[j] if j < len(self.t) else ("eof", "", self.t[-1][2] if self.t else 0)

    def take(self, kind: str | None = None, value: str | None = None):
        tok = self.peek()
        if (kind and tok[0] != kind) or (value is not None and tok[1] != value):
            want = value or kind
            raise IdlError(f"expected {want}, got {tok[1] or tok[0]!r}", tok[2])
        self.i += 1
        return tok

    def type_(self) -> str:
        name = self.take("name")[1]
        if self.peek()[1] == "<":
            self.take("punct", "<")
            params = [self.type_()]
            while self.peek()[1] == ",":
                self.take("punct", ",")
                params.append(self.type_())
            self.take("punct", ">")
            return f"{name}<{','.join(params)}>"
        return name

    def fields(self, close: str) -> list[Field]:
        out = []
        while self.peek()[1] != close:
            idx = int(self.take("int")[1])
            self.take("punct", ":")
            ty = self.type_()
            nm = self.take("name")[1]
            out.append(Field(idx, ty, nm))
            if self.peek()[1] == ",":
                self.take("punct", ",")
        return out

    def parse(self) -> IdlFile:
        f = IdlFile()
        docs: list[str] = []
        while self.peek()[0] != "eof":
            kind, v, line = self.peek()
            if kind in ("doc", "deco"):   # stray top-level doc / decorator lines
                self.i += 1
                continue
            if v in ("message", "exception"):
                self.take()
                name = self.take("name")[1]
                native = ""
                if self.peek()[1] == "(":
                    self.take("punct", "(")
                    native = self.take("string")[1].strip('"')
                    self.take("punct", ")")
                self.take("punct", "{")
                flds = self.fields("}")
                self.take("punct", "}")
                f.messages.append(Message(name, flds, native, v == "exception"))
            elif v == "type":
                self.take()
                name = self.take("name")[1]
                self.take("punct", "=")
                f.typedefs[name] = self.type_()
            elif v == "enum":
                self.take()
                name = self.take("name")[1]
                self.take("punct", "{")
                vals = []
                while self.peek()[1] != "}":
                    n = int(self.take("int")[1])
                    self.take("punct", ":")
                    vals.append((n, self.take("name")[1]))
                self.take("punct", "}")
                f.enums[name] = vals
            elif v == "service":
                self.take()
                name = self.take("name")[1]
                self.take("punct", "{")
                f.services.append(Service(name, self.methods()))
                self.take("punct", "}")
            else:
                raise IdlError(f"unexpected {v!r}", line)
        del docs
        return f

    def methods(self) -> list[IdlMethod]:
        out = []
        doc: list[str] = []
        decos: list[tuple[str, int]] = []
        while self.peek()[1] != "}":
            kind, v, line = self.peek()
            if kind == "doc":
                self.i += 1
                doc.append(v[2:].rstrip())
                continue
            if kind == "deco":
                self.i += 1
                decos.append((v[2:], line))
                continue
            ret = self.type_()
            name = self.take("name")[1]
            self.take("punct", "(")
            args = self.fields(")")
            self.take("punct", ")")
            m = IdlMethod(name, ret, args, doc=_dedent(doc))
            seen = set()
            for d, dl in decos:
                base, _, num = d.partition("(")
                if base in ROUTINGS:
                    m.routing = base
                    if base == "cht":
                        m.cht_n = int(num.rstrip(")").strip()) if num else 2
                    seen.add("routing")
                elif base in LOCKS:
                    m.lock = base
                    seen.add("lock")
                elif base in AGGS:
                    m.agg = base
                    seen.add("agg")
                else:
                    raise IdlError(f"unknown decorator #@{d}", dl)
            if "routing" not in seen or "lock" not in seen:
                raise IdlError(f"method {name} needs a routing and a request-type decorator", line)
            out.append(m)
            doc, decos = [], []
        return out


def _dedent(lines: list[str]) -> list[str]:
    strip = [ln[1:] if ln.startswith(" ") else ln for ln in lines]
    return strip


def parse(text: str) -> IdlFile:
    return _Parser(tokenize(text)).parse()


def parse_file(path: str) -> IdlFile:
    with open(path, encoding="utf-8") as fp:
        return parse(fp.read())


def norm_type(t: str) -> str:
    return re.sub(r"\s+", "", t)
