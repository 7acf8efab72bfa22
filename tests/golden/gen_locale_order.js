// Golden vectors for String.prototype.localeCompare, the collation
// RiskAnalyzer.Impact sorts service names with (RiskAnalyzer.ts:57-60).
// Run with the Node that runs the reference (node 12.22.9, ICU 70.1, en-US):
//   node tests/golden/gen_locale_order.js > tests/golden/locale_order.json
// Emits the corpus sorted by localeCompare (V8's sort is stable), the
// comparison sign of every adjacent pair, and the collation tables it probed
// (whitespace / punctuation order, the secondary order of combining marks).
"use strict";
const corpus = [];
const svc = ["reviews", "Reviews", "ratings", "details", "product-page", "product_page", "productpage",
  "productPage", "prod.page", "svc-01", "svc-1", "svc-10", "svc-2", "svc_01", "SVC-01", "a", "A", "ab", "a-b",
  "a_b", "a.b", "a b", "a\tb", "a\nb", "a\u0001b", "a:b", "a/b", "a@b", "a$b", "a~b", "a+b", "café", "cafe",
  "Café", "cafè", "caff", "niño", "nino", "über", "uber", "Über", "öl", "ol", "zeta", "Zeta", "é", "é",
  "1abc", "10abc", "9abc", "_x", "-x", ".x", "x", "X"];
const ns = ["default", "book-info", "bookinfo", "prod", "Prod"];
const ver = ["v1", "v2", "v10", "latest", "undefined"];
for (const s of svc) corpus.push(s);
for (const s of svc.slice(0, 20)) for (const n of ns) for (const v of ver) corpus.push(`${s}\t${n}\t${v}`);
const sorted = corpus.slice().sort((a, b) => a.localeCompare(b));
const signs = [];
for (let i = 1; i < sorted.length; i++) signs.push(Math.sign(sorted[i - 1].localeCompare(sorted[i])));
const punct = [];
for (let i = 0; i < 127; i++) {
  const c = String.fromCharCode(i);
  if (!/[A-Za-z0-9]/.test(c)) punct.push(c);
}
const marks = [];
for (let m = 0x300; m <= 0x36f; m++) marks.push("e" + String.fromCharCode(m));
const markOrder = marks.slice().sort((a, b) => a.localeCompare(b));
const markSigns = [];
for (let i = 1; i < markOrder.length; i++) markSigns.push(Math.sign(markOrder[i - 1].localeCompare(markOrder[i])));
process.stdout.write(JSON.stringify({
  node: process.version, icu: process.versions.icu, locale: Intl.Collator().resolvedOptions().locale,
  corpus, sorted, signs,
  punct_sorted: punct.slice().sort((a, b) => a.localeCompare(b)),
  punct_ignorable: punct.filter((c) => ("a" + c + "b").localeCompare("ab") === 0),
  marks_sorted: markOrder.map((x) => x.charCodeAt(1)), marks_signs: markSigns,
}, null, 0) + "\n");
