// node tests/js/embed_test.js -- pym-protocol parent/child exchange over a fake DOM.
"use strict";
const fs = require("fs");
const path = require("path");
const vm = require("vm");
const src = fs.readFileSync(path.join(__dirname, "../../twitter_stream_ml_amd/web/assets/js/embed.js"), "utf8");

function fakeWindow(name, search) {
  const listeners = {};
  const w = {
    name, listeners, sent: [],
    location: { href: "http://dash.local/index.html", search: search || "" },
    addEventListener(t, fn) { (listeners[t] = listeners[t] || []).push(fn); },
    removeEventListener(t, fn) { listeners[t] = (listeners[t] || []).filter((f) => f !== fn); },
    dispatch(t, ev) { (listeners[t] || []).slice().forEach((f) => f(ev)); },
    setInterval() {},
  };
  // a real postMessage reports the sending window as ev.source: w.peer
  w.postMessage = (data) => { w.sent.push(data); w.dispatch("message", { data, origin: "http://dash.local", source: w.peer }); };
  return w;
}

function makeDocument(win, bodyHeight) {
  const els = {};
  const doc = {
    readyState: "complete",
    location: { href: "" },
    getElementById: (id) => els[id],
    getElementsByTagName: () => [{ offsetHeight: bodyHeight }],
    querySelectorAll: () => [],
    addEventListener() {},
    createElement: () => {
      const attrs = {}, evl = {};
      return { attrs, evl, setAttribute: (k, v) => { attrs[k] = v; },
               addEventListener: (t, fn) => { evl[t] = fn; }, parentNode: null, contentWindow: null };
    },
  };
  doc.els = els;
  win.document = doc;
  return doc;
}

function load(win) {
  const ctx = { window: win, document: win.document };
  vm.runInNewContext(src, ctx);
  return win.embed;
}

let failures = 0;
function check(cond, what) { if (!cond) { failures++; console.error("FAIL:", what); } }

// parent page
const pw = fakeWindow("parent");
const pdoc = makeDocument(pw, 0);
const container = { offsetWidth: 640, appendChild(f) { f.parentNode = this; this.frame = f; },
                    removeChild(f) { f.parentNode = null; } };
pdoc.els.viz1 = container;
const P = load(pw);
const parent = new P.Parent("viz1", "http://lgn.local/visualizations/7/pym#top");
const src0 = parent.iframe.src;
check(src0 === "http://lgn.local/visualizations/7/pym?initialWidth=640&childId=viz1&parentUrl=" +
      encodeURIComponent("http://dash.local/index.html") + "#top", "iframe src " + src0);
check(parent.iframe.attrs.scrolling === "no" && parent.iframe.attrs.width === "100%", "iframe attrs");

// child page inside the iframe
const cw = fakeWindow("child", "?initialWidth=640&childId=viz1&parentUrl=x");
makeDocument(cw, 321);
cw.parent = pw;                       // child -> parent messages
parent.iframe.contentWindow = cw;     // parent -> child messages
pw.peer = cw; cw.peer = pw;
const C = load(cw);
let rendered = [];
const child = new C.Child({ renderCallback: (w) => rendered.push(w) });
check(child.id === "viz1" && child.parentWidth === 640, "child query parse");
check(rendered[0] === 640, "initial render");
check(parent.iframe.attrs.height === "321px", "height on child load: " + parent.iframe.attrs.height);

// parent load + resize -> width -> child re-renders and answers with its height
container.offsetWidth = 480;
cw.document.getElementsByTagName = () => [{ offsetHeight: 555 }];
parent.iframe.evl.load();
check(rendered[rendered.length - 1] === 480, "width on load");
check(parent.iframe.attrs.height === "555px", "height after width");
container.offsetWidth = 300;
pw.dispatch("resize", {});
check(child.parentWidth === 300, "width on resize");
check(cw.sent.some((m) => m === "pymxPYMxviz1xPYMxwidthxPYMx300"), "wire format");

// navigateTo; messages for another id or non-strings are ignored
child.navigateParentTo("http://elsewhere/");
check(pw.document.location.href === "http://elsewhere/", "navigateTo");
child.scrollParentTo("sec2");
check(pw.document.location.href === "#sec2", "navigateTo fragment");
// script / data URLs (even disguised) never reach location.href
for (const bad of ["javascript:alert(1)", " javascript:alert(1)", "java\tscript:alert(1)", "JAVASCRIPT:x",
                   "data:text/html,<script>1</script>", "vbscript:x", "//evil.example/", "http:/x"]) {
  child.navigateParentTo(bad);
  check(pw.document.location.href === "#sec2", "navigateTo blocked: " + JSON.stringify(bad));
}
// a message from some other window (not our iframe) is ignored even if well formed
pw.dispatch("message", { data: "pymxPYMxviz1xPYMxnavigateToxPYMxhttp://phish.example/", origin: "http://dash.local",
                         source: { other: true } });
check(pw.document.location.href === "#sec2", "foreign source ignored");
pw.dispatch("message", { data: "pymxPYMxviz1xPYMxheightxPYMx9", origin: "http://dash.local", source: undefined });
check(parent.iframe.attrs.height !== "9px", "sourceless message ignored");
const h0 = parent.iframe.attrs.height;
pw.dispatch("message", { data: "pymxPYMxotherxPYMxheightxPYMx1", origin: "x" });
pw.dispatch("message", { data: { obj: 1 }, origin: "x" });
check(parent.iframe.attrs.height === h0, "foreign messages ignored");
check(P._parse("viz1", "pymxPYMxviz1xPYMxbad typexPYMx1") === null, "type without spaces");

// xdomain filter
const strict = new P.Parent("viz1", "http://lgn.local/v", { xdomain: "lgn\\.local" });
strict.iframe.contentWindow = cw;
pw.dispatch("message", { data: "pymxPYMxviz1xPYMxheightxPYMx99", origin: "http://evil.example", source: cw });
check(strict.iframe.attrs.height !== "99px", "xdomain blocks");
pw.dispatch("message", { data: "pymxPYMxviz1xPYMxheightxPYMx77", origin: "http://lgn.local:3000", source: cw });
check(strict.iframe.attrs.height === "77px", "xdomain allows");
strict.remove();

if (failures) { console.error(failures + " failure(s)"); process.exit(1); }
console.log("embed.js ok");
