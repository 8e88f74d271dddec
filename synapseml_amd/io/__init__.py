"""IO: HTTP on DataFrames, batched serving, binary files, PowerBI writer
(reference: core/.../io/**, SPX/sql/execution/streaming/**)."""
from .binary import BinaryFileFields, read_binary_files, write_binary_files, zip_bytes
from .http import (CustomInputParser, CustomOutputParser, HTTPTransformer, JSONInputParser, JSONOutputParser,
                   SimpleHTTPTransformer, StringOutputParser, advanced_handler, basic_handler, make_request,
                   response_string, send_with_retries)
from .powerbi import PowerBIWriter
from .serving import ServingServer, make_reply, make_response, parse_request, request_to_string, serve
from .streaming import ContinuousServingServer, ServingQuery, read_stream

__all__ = ["ContinuousServingServer", "ServingQuery", "read_stream", "BinaryFileFields", "read_binary_files", "write_binary_files", "zip_bytes", "HTTPTransformer",
           "SimpleHTTPTransformer", "JSONInputParser", "JSONOutputParser", "StringOutputParser",
           "CustomInputParser", "CustomOutputParser", "advanced_handler", "basic_handler", "make_request",
           "response_string", "send_with_retries", "PowerBIWriter", "ServingServer", "serve", "parse_request",
           "make_reply", "make_response", "request_to_string"]
