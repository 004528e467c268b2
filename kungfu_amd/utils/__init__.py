from .._utils import EMA, _log_event, map_maybe, measure, show_duration
