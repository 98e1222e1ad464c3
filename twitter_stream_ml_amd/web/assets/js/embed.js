/* Minimal responsive-iframe parent for Lightning's /visualizations/<id>/pym
 * pages: the child posts "xPYMx"-delimited "height" messages (pym.js
 * protocol); we resize the iframe accordingly. */
(function (global) {
  "use strict";
  function Parent(containerId, url) {
    var el = document.getElementById(containerId);
    var frame = document.createElement("iframe");
    var id = containerId;
    frame.src = url + (url.indexOf("?") < 0 ? "?" : "&") + "initialWidth=" + el.offsetWidth +
                "&childId=" + encodeURIComponent(id);
    frame.setAttribute("scrolling", "no");
    el.appendChild(frame);
    global.addEventListener("message", function (ev) {
      if (typeof ev.data !== "string") return;
      var parts = ev.data.split("xPYMx");
      if (parts.length === 4 && parts[1] === id && parts[2] === "height") {
        frame.style.height = parseInt(parts[3], 10) + "px";
      }
    });
    this.iframe = frame;
  }
  global.embed = { Parent: Parent };
})(window);
