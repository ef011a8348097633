from .summary import BasicStatisticalSummary
