"""Stand-in for the absent web.parms module imported by bin/inference.py:26."""


class GlobalParams:
    def __init__(self, *args, **kwargs):
        self.args, self.kwargs = args, kwargs
