"""Diagnostic report rendering (text and self-contained HTML with inline SVG plots).

Reference: ``photon-diagnostics/.../reporting/**`` — a logical report (system report: parameters, feature
summary; one model report per λ: metrics, Hosmer–Lemeshow, prediction/error independence, feature importance,
fitting curves, bootstrap) is transformed into a physical document of chapters / sections / text / bullet lists /
tables / plots, and rendered with an HTML strategy (xchart plots embedded as SVG) or a text strategy.
``Driver.diagnose`` writes ``<output>/diagnostic.html`` (the reference: ``model-diagnostic.html``).

Here the physical document is a small tree of :class:`Chapter`/:class:`Section` objects holding
strings, tables and :class:`Plot` items; plots are rendered directly to SVG (no plotting library needed).
"""
from __future__ import annotations

import html
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple, Union


@dataclass
class Plot:
    title: str
    x_label: str
    y_label: str
    series: List[Tuple[str, Sequence[float], Sequence[float]]]  # (name, xs, ys)
    kind: str = "line"  # line | bar

    def svg(self, w: int = 560, h: int = 320) -> str:
        pad_l, pad_r, pad_t, pad_b = 60, 120, 30, 40
        xs = [float(x) for _, sx, _ in self.series for x in sx]
        ys = [float(y) for _, _, sy in self.series for y in sy if math.isfinite(float(y))]
        if not xs or not ys:
            return f"<p>(no data for {html.escape(self.title)})</p>"
        x0, x1 = min(xs), max(xs)
        y0, y1 = min(ys + [0.0]) if self.kind == "bar" else min(ys), max(ys)
        if x1 == x0:
            x1 = x0 + 1
        if y1 == y0:
            y1 = y0 + 1

        def px(x):
            return pad_l + (float(x) - x0) / (x1 - x0) * (w - pad_l - pad_r)

        def py(y):
            return h - pad_b - (float(y) - y0) / (y1 - y0) * (h - pad_t - pad_b)
        colors = ["#1f77b4", "#d62728", "#2ca02c", "#ff7f0e", "#9467bd", "#8c564b"]
        out = [f'<svg xmlns="http://www.w3.org/2000/svg" width="{w}" height="{h}" font-size="11">',
               f'<text x="{w / 2}" y="16" text-anchor="middle" font-weight="bold">{html.escape(self.title)}</text>',
               f'<line x1="{pad_l}" y1="{h - pad_b}" x2="{w - pad_r}" y2="{h - pad_b}" stroke="black"/>',
               f'<line x1="{pad_l}" y1="{pad_t}" x2="{pad_l}" y2="{h - pad_b}" stroke="black"/>',
               f'<text x="{(w - pad_r + pad_l) / 2}" y="{h - 8}" text-anchor="middle">{html.escape(self.x_label)}</text>',
               f'<text x="14" y="{(h - pad_b + pad_t) / 2}" transform="rotate(-90 14 {(h - pad_b + pad_t) / 2})" '
               f'text-anchor="middle">{html.escape(self.y_label)}</text>']
        for t in range(5):
            yv = y0 + (y1 - y0) * t / 4
            out.append(f'<text x="{pad_l - 4}" y="{py(yv) + 4}" text-anchor="end">{yv:.3g}</text>')
            xv = x0 + (x1 - x0) * t / 4
            out.append(f'<text x="{px(xv)}" y="{h - pad_b + 14}" text-anchor="middle">{xv:.3g}</text>')
        n_series = max(1, len(self.series))
        for si, (name, sx, sy) in enumerate(self.series):
            c = colors[si % len(colors)]
            if self.kind == "bar":
                bw = max(1.0, (w - pad_l - pad_r) / max(1, len(sx)) / n_series * 0.8)
                for x, y in zip(sx, sy):
                    xx = px(x) + si * bw
                    out.append(f'<rect x="{xx:.1f}" y="{min(py(y), py(0)):.1f}" width="{bw:.1f}" '
                               f'height="{abs(py(0) - py(y)):.1f}" fill="{c}"/>')
            else:
                pts = " ".join(f"{px(x):.1f},{py(y):.1f}" for x, y in zip(sx, sy) if math.isfinite(float(y)))
                out.append(f'<polyline fill="none" stroke="{c}" stroke-width="1.5" points="{pts}"/>')
            out.append(f'<text x="{w - pad_r + 8}" y="{pad_t + 14 * (si + 1)}" fill="{c}">{html.escape(name)}</text>')
        out.append("</svg>")
        return "".join(out)

    def text(self) -> str:
        lines = [f"[plot] {self.title} ({self.x_label} vs {self.y_label})"]
        for name, sx, sy in self.series:
            lines.append(f"  {name}: " + ", ".join(f"({float(x):.4g}, {float(y):.4g})" for x, y in zip(sx, sy)))
        return "\n".join(lines)


@dataclass
class Table:
    header: List[str]
    rows: List[List[object]]


Item = Union[str, List[str], Table, Plot]


@dataclass
class Section:
    title: str
    items: List[Item] = field(default_factory=list)


@dataclass
class Chapter:
    title: str
    sections: List[Section] = field(default_factory=list)


@dataclass
class Document:
    title: str
    chapters: List[Chapter] = field(default_factory=list)

    # ---------------------------------------------------------------- renderers
    def to_text(self) -> str:
        out = [self.title, "=" * len(self.title), ""]
        for ci, ch in enumerate(self.chapters, 1):
            out += [f"{ci}. {ch.title}", "-" * (len(ch.title) + 4)]
            for si, sec in enumerate(ch.sections, 1):
                out.append(f"{ci}.{si} {sec.title}")
                for it in sec.items:
                    out.append(_item_text(it))
                out.append("")
        return "\n".join(out)

    def to_html(self) -> str:
        out = ["<!DOCTYPE html><html><head><meta charset='utf-8'>",
               f"<title>{html.escape(self.title)}</title>",
               "<style>body{font-family:sans-serif;max-width:1100px;margin:auto}table{border-collapse:collapse}"
               "td,th{border:1px solid #999;padding:2px 6px;font-size:12px}pre{background:#f4f4f4;padding:6px}"
               "</style></head><body>", f"<h1>{html.escape(self.title)}</h1>"]
        out.append("<ol>" + "".join(f"<li><a href='#ch{i}'>{html.escape(c.title)}</a></li>"
                                    for i, c in enumerate(self.chapters, 1)) + "</ol>")
        for ci, ch in enumerate(self.chapters, 1):
            out.append(f"<h2 id='ch{ci}'>{ci}. {html.escape(ch.title)}</h2>")
            for si, sec in enumerate(ch.sections, 1):
                out.append(f"<h3>{ci}.{si} {html.escape(sec.title)}</h3>")
                out += [_item_html(it) for it in sec.items]
        out.append("</body></html>")
        return "\n".join(out)


def _item_text(it: Item) -> str:
    if isinstance(it, str):
        return it
    if isinstance(it, list):
        return "\n".join(f"  * {x}" for x in it)
    if isinstance(it, Table):
        widths = [max(len(str(h)), *(len(_fmt(r[i])) for r in it.rows)) if it.rows else len(str(h))
                  for i, h in enumerate(it.header)]
        lines = [" | ".join(str(h).ljust(w) for h, w in zip(it.header, widths))]
        lines.append("-+-".join("-" * w for w in widths))
        lines += [" | ".join(_fmt(c).ljust(w) for c, w in zip(r, widths)) for r in it.rows]
        return "\n".join(lines)
    return it.text()


def _item_html(it: Item) -> str:
    if isinstance(it, str):
        return f"<pre>{html.escape(it)}</pre>" if "\n" in it else f"<p>{html.escape(it)}</p>"
    if isinstance(it, list):
        return "<ul>" + "".join(f"<li>{html.escape(str(x))}</li>" for x in it) + "</ul>"
    if isinstance(it, Table):
        head = "".join(f"<th>{html.escape(str(h))}</th>" for h in it.header)
        body = "".join("<tr>" + "".join(f"<td>{html.escape(_fmt(c))}</td>" for c in r) + "</tr>" for r in it.rows)
        return f"<table><tr>{head}</tr>{body}</table>"
    return it.svg()


def _fmt(v) -> str:
    if isinstance(v, float):
        return f"{v:.6g}"
    return str(v)


# ------------------------------------------------------------------------------------------------ transformers
def system_chapter(params: Optional[dict], index_map=None, summary=None, max_features: int = 50) -> Chapter:
    secs = []
    if params:
        secs.append(Section("Parameters", [Table(["parameter", "value"], [[k, v] for k, v in sorted(params.items())])]))
    if summary is not None:
        d = len(summary.mean)
        rows = []
        for j in range(min(d, max_features)):
            name = index_map.get_feature_name(j) if index_map is not None else str(j)
            rows.append([str(name).replace("\u0001", ":"), float(summary.mean[j]), float(summary.variance[j]),
                         float(summary.min[j]), float(summary.max[j]), int(summary.num_nonzeros[j])])
        secs.append(Section(f"Feature summary ({summary.count} samples, {d} features; first {len(rows)} shown)",
                            [Table(["feature", "mean", "variance", "min", "max", "nnz"], rows)]))
    return Chapter("System", secs)


def model_chapter(rep) -> Chapter:
    secs = [Section("Metrics", [Table(["metric", "value"], [[k, v] for k, v in sorted(rep.metrics.items())])])]
    if rep.hosmer_lemeshow is not None:
        hl = rep.hosmer_lemeshow
        b = hl.histogram
        centres = [0.5 * (x.lower + x.upper) for x in b]
        secs.append(Section("Hosmer-Lemeshow goodness of fit", [
            hl.test_description(), hl.point_probability(), hl.binning_msg,
            Plot("Observed vs expected positives per probability bin", "predicted probability", "count",
                 [("observed", centres, [x.observed_pos for x in b]),
                  ("expected", centres, [x.expected_pos for x in b])], kind="bar")]
            + ([hl.chi_square_msg] if hl.chi_square_msg else [])))
    if rep.prediction_error_independence is not None:
        kt = rep.prediction_error_independence.kendall_tau
        secs.append(Section("Prediction / error independence (Kendall tau)", [[
            f"tau-alpha = {kt.tau_alpha:.6g}", f"tau-beta = {kt.tau_beta:.6g}", f"z = {kt.z_alpha:.6g}",
            f"p-value = {kt.p_value:.6g}", f"concordant = {kt.concordant}, discordant = {kt.discordant}, "
                                            f"items = {kt.n_items}"]] + ([kt.message] if kt.message else [])))
    for imp in (rep.mean_impact_importance, rep.variance_impact_importance):
        if imp is None:
            continue
        rows = [[f"{k[0]}:{k[1]}", v[0], v[1]] for k, v in sorted(imp.feature_importance.items(),
                                                                  key=lambda kv: -kv[1][1])]
        fr = sorted(imp.rank_to_importance.items())
        secs.append(Section(f"Feature importance: {imp.importance_type}", [
            imp.importance_description, Table(["feature", "index", "importance"], rows),
            Plot("Importance by rank fractile", "fractile (%)", "importance",
                 [("importance", [f for f, _ in fr], [v for _, v in fr])])]))
    if rep.fit_report is not None:
        items: List[Item] = [rep.fit_report.message] if rep.fit_report.message else []
        for metric, (portion, train, test) in sorted(rep.fit_report.metrics.items()):
            items.append(Plot(f"Learning curve: {metric}", "training portion (%)", metric,
                              [("train", portion, train), ("hold-out", portion, test)]))
        secs.append(Section("Fitting diagnostic", items))
    if rep.bootstrap_report is not None:
        br = rep.bootstrap_report
        rows = [[k, *v] for k, v in sorted(br.metric_distributions.items())]
        secs.append(Section("Bootstrap", [
            Table(["metric", "min", "Q1", "median", "Q3", "max"], rows),
            "Important features: " + ", ".join(f"{k[0]}:{k[1]} {v}" for k, v in br.important_features.items()),
            f"{len(br.zero_crossing_features)} coefficient(s) with an inter-quartile range straddling 0"]))
    return Chapter(rep.description, secs)


def build_document(title: str, model_reports, params=None, index_map=None, summary=None) -> Document:
    return Document(title, [system_chapter(params, index_map, summary)] + [model_chapter(r) for r in model_reports])
