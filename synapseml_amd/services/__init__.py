"""Cognitive-service transformers over HTTP (reference: cognitive/.../services/**).

Every transformer builds one request per row from scalar or per-column
``ServiceParam`` values, sends them concurrently with retries, polls async
operations and returns parsed JSON in ``outputCol`` / failures in ``errorCol``."""
from .anomaly import (DetectAnomalies, DetectLastAnomaly, DetectLastMultivariateAnomaly, DetectMultivariateAnomaly,
                      SimpleDetectAnomalies, SimpleDetectMultivariateAnomaly, SimpleFitMultivariateAnomaly)
from .base import CognitiveServicesBase, HasAsyncReply, ServiceParam, ServiceValue
from .form import (AnalyzeBusinessCards, AnalyzeCustomModel, AnalyzeDocument, AnalyzeIDDocuments, AnalyzeInvoices,
                   AnalyzeLayout, AnalyzeReceipts, FormOntologyLearner, FormOntologyTransformer, GetCustomModel,
                   ListCustomModels)
from .langchain import LangchainTransformer
from .misc import (AddDocuments, AddressGeocoder, AzureSearchWriter, BingImageSearch, CheckPointInPolygon,
                   ConversationTranscription,
                   ReverseAddressGeocoder, SpeakerEmotionInference, SpeechToText, SpeechToTextSDK, TextToSpeech)
from .openai import OpenAIChatCompletion, OpenAICompletion, OpenAIDefaults, OpenAIEmbedding, OpenAIPrompt
from .text import (NER, PII, AnalyzeHealthText, AnalyzeText, TextAnalyze, BreakSentence, Detect, DictionaryExamples,
                   DictionaryLookup, DocumentTranslator, EntityDetector, KeyPhraseExtractor, LanguageDetector,
                   TextSentiment, Translate, Transliterate)
from .vision import (OCR, AnalyzeImage, DescribeImage, DetectFace, FindSimilarFace, GenerateThumbnails, GroupFaces,
                     IdentifyFaces, ReadImage, RecognizeDomainSpecificContent, RecognizeText, TagImage, VerifyFaces)

__all__ = [n for n in dir() if not n.startswith("_")]
