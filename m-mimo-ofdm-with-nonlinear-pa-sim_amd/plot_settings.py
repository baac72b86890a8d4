"""Matplotlib style of the reference (plot_settings.py) -- cosmetic, out of scope.
Kept as a no-op so unmodified drivers that call it still import and run headless."""


def set_latex_plot_style(use_tex: bool = False, fig_width_in: float = 7.0, fig_height_in: float = None) -> None:
    return None
