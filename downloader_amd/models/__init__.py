"""Wire models of the staging service: protobuf messages (``api``) and the S3 layout."""
from . import api, keys  # noqa: F401
from .api import (Convert, Download, Media, TelemetryProgress, TelemetryStatus,  # noqa: F401
                  STATUS_DOWNLOADING, STATUS_ERRORED)
