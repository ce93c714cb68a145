from .load_data import (IndexReturnsRetriever, RollingWindows, SharedCacheIndexReturns, centred_series,  # noqa: F401
                        load_returns_csv, returns_from_prices)
