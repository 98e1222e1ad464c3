/* Responsive iframe embedding, wire-compatible with pym.js 0.4.5 (the
 * library the reference dashboard vendors, web/src/main/assets/lib/pym/pym.js:
 * Parent :132-364, Child :372-585), so Lightning's /visualizations/<id>/pym
 * child pages size themselves inside the dashboard.
 *
 * Protocol: window.postMessage strings "pym" xPYMx <id> xPYMx <type> xPYMx
 * <message>.  The parent creates the iframe with ?initialWidth=&childId=
 * &parentUrl= (fragment kept) and sends "width" when the iframe loads and
 * on every resize; the child sends "height" (its document height) on load, on
 * resize and after every width message, and "navigateTo" to move the parent
 * page.  Messages whose origin does not match the xdomain setting (a regex
 * source, default any) are ignored, and so are messages not sent by the
 * iframe's own window (parent side) or by the parent window (child side).
 * Unlike pym.js 0.4.5 (pym.js:254-256, which assigns any string to
 * location.href -- a "javascript:" URL runs in the dashboard's origin),
 * "navigateTo" only accepts a "#fragment" or an absolute http(s) URL.
 * Exposed as window.embed and window.pym.
 */
(function (global) {
  "use strict";

  var SEP = "xPYMx";

  function frame(id, type, message) {
    return ["pym", id, type, message].join(SEP);
  }

  function parse(id, data) {
    // -> [type, message] for a message addressed to `id`, else null
    if (typeof data !== "string") return null;
    var head = "pym" + SEP + id + SEP;
    if (data.indexOf(head) !== 0) return null;
    var rest = data.substring(head.length);
    var cut = rest.indexOf(SEP);
    if (cut <= 0) return null;
    var type = rest.substring(0, cut), message = rest.substring(cut + SEP.length);
    if (/\s/.test(type) || message.length === 0) return null;
    return [type, message];
  }

  function originOk(ev, xdomain) {
    if (!xdomain || xdomain === "*") return true;
    return new RegExp("^https?://" + xdomain + "(:\\d+)?$").test(ev.origin);
  }

  function safeNavTarget(m) {
    // no whitespace / control characters (browsers strip them out of schemes)
    if (/[\u0000-\u0020\u007f]/.test(m)) return false;
    return /^#/.test(m) || /^https?:\/\/[^\/]/i.test(m);
  }

  function Handlers() { this.map = {}; }
  Handlers.prototype.on = function (type, fn) { (this.map[type] = this.map[type] || []).push(fn); };
  Handlers.prototype.fire = function (self, type, message) {
    var list = this.map[type] || [];
    for (var i = 0; i < list.length; i++) list[i].call(self, message);
  };

  /* Parent: renders `url` as an iframe into the element with id `id`. */
  function Parent(id, url, config) {
    var self = this;
    this.id = id;
    this.el = document.getElementById(id);
    this.settings = { xdomain: "*" };
    for (var k in (config || {})) this.settings[k] = config[k];
    this.handlers = new Handlers();

    var hash = "", at = url.indexOf("#");
    if (at >= 0) { hash = url.substring(at); url = url.substring(0, at); }
    this.url = url;
    this.iframe = document.createElement("iframe");
    this.iframe.src = url + (url.indexOf("?") < 0 ? "?" : "&") +
      "initialWidth=" + this.el.offsetWidth +
      "&childId=" + id +
      "&parentUrl=" + encodeURIComponent(global.location.href) + hash;
    this.iframe.setAttribute("width", "100%");
    this.iframe.setAttribute("scrolling", "no");
    this.iframe.setAttribute("marginheight", "0");
    this.iframe.setAttribute("frameborder", "0");

    this.onMessage("height", function (m) {
      self.iframe.setAttribute("height", parseInt(m, 10) + "px");
    });
    this.onMessage("navigateTo", function (m) { if (safeNavTarget(m)) global.document.location.href = m; });

    this._onMessage = function (ev) {
      if (!originOk(ev, self.settings.xdomain)) return;
      if (ev.source !== self.iframe.contentWindow) return;   // only our own iframe
      var m = parse(self.id, ev.data);
      if (m) self.handlers.fire(self, m[0], m[1]);
    };
    this._onResize = function () { self.sendWidth(); };
    global.addEventListener("message", this._onMessage, false);
    global.addEventListener("resize", this._onResize, false);
    this.el.appendChild(this.iframe);
    this.iframe.addEventListener("load", this._onResize, false);
  }
  Parent.prototype.onMessage = function (type, fn) { this.handlers.on(type, fn); };
  Parent.prototype.sendMessage = function (type, message) {
    if (this.iframe.contentWindow) this.iframe.contentWindow.postMessage(frame(this.id, type, message), "*");
  };
  Parent.prototype.sendWidth = function () { this.sendMessage("width", String(this.el.offsetWidth)); };
  Parent.prototype.remove = function () {
    global.removeEventListener("message", this._onMessage);
    global.removeEventListener("resize", this._onResize);
    if (this.iframe.parentNode) this.iframe.parentNode.removeChild(this.iframe);
  };

  /* Child: the embedded page's half; config.renderCallback(width) redraws. */
  function Child(config) {
    var self = this;
    this.settings = { renderCallback: null, xdomain: "*", polling: 0 };
    for (var k in (config || {})) this.settings[k] = config[k];
    this.handlers = new Handlers();
    var q = {};
    var qs = global.location.search.replace(/^\?/, "").split("&");
    for (var i = 0; i < qs.length; i++) {
      var kv = qs[i].split("=");
      if (kv[0]) q[decodeURIComponent(kv[0])] = decodeURIComponent(kv.slice(1).join("="));
    }
    this.id = q.childId || this.settings.id || "";
    this.parentUrl = q.parentUrl || "";
    this.parentWidth = q.initialWidth ? parseInt(q.initialWidth, 10) : null;

    this.onMessage("width", function (m) {
      self.parentWidth = parseInt(m, 10);
      if (self.settings.renderCallback) self.settings.renderCallback(self.parentWidth);
      self.sendHeight();
    });
    this._onMessage = function (ev) {
      if (!originOk(ev, self.settings.xdomain)) return;
      if (ev.source !== global.parent) return;                // only the embedding page
      var m = parse(self.id, ev.data);
      if (m) self.handlers.fire(self, m[0], m[1]);
    };
    global.addEventListener("message", this._onMessage, false);
    global.addEventListener("resize", function () { self.sendHeight(); }, false);
    if (this.settings.renderCallback && this.parentWidth) this.settings.renderCallback(this.parentWidth);
    this.sendHeight();
    if (this.settings.polling > 0) global.setInterval(function () { self.sendHeight(); }, this.settings.polling);
  }
  Child.prototype.onMessage = function (type, fn) { this.handlers.on(type, fn); };
  Child.prototype.sendMessage = function (type, message) {
    if (global.parent && global.parent !== global) global.parent.postMessage(frame(this.id, type, message), "*");
  };
  Child.prototype.sendHeight = function () {
    var h = global.document.getElementsByTagName("body")[0].offsetHeight;
    this.sendMessage("height", String(h));
  };
  Child.prototype.scrollParentTo = function (hash) { this.sendMessage("navigateTo", "#" + hash); };
  Child.prototype.navigateParentTo = function (url) { this.sendMessage("navigateTo", url); };

  /* data-pym-src elements become parents once the page has loaded. */
  function autoInit() {
    var els = global.document.querySelectorAll("[data-pym-src]:not([data-pym-auto-initialized])");
    for (var i = 0; i < els.length; i++) {
      var el = els[i];
      el.setAttribute("data-pym-auto-initialized", "");
      if (!el.id) el.id = "pym-" + i;
      var xd = el.getAttribute("data-pym-xdomain");
      new Parent(el.id, el.getAttribute("data-pym-src"), xd ? { xdomain: xd } : {});
    }
  }

  var api = { Parent: Parent, Child: Child, autoInit: autoInit, _frame: frame, _parse: parse,
              _safeNavTarget: safeNavTarget };
  global.embed = api;
  if (!global.pym) global.pym = api;
  if (global.document && global.document.readyState !== "loading") autoInit();
  else if (global.document) global.document.addEventListener("DOMContentLoaded", autoInit);
})(window);
