"""Computer Vision and Face transformers (reference:
cognitive/.../services/vision/ComputerVision.scala:33-650, face/Face.scala).

Images are given either as a URL (``imageUrl``) — sent as ``{"url": ...}``
— or as raw bytes (``imageBytes``) — sent as application/octet-stream."""
from __future__ import annotations

import json

from .base import CognitiveServicesBase, HasAsyncReply, ServiceParam


class _ImageInput(CognitiveServicesBase):
    imageUrl = ServiceParam("the url of the image to use")
    imageBytes = ServiceParam("bytestream of the image to use")

    def _should_skip(self, vals):
        return vals.get("imageUrl") is None and vals.get("imageBytes") is None

    def _entity(self, vals):
        if vals.get("imageBytes") is not None:
            return bytes(vals["imageBytes"]), "application/octet-stream"
        return json.dumps({"url": vals["imageUrl"]}).encode("utf-8"), "application/json"


class AnalyzeImage(_ImageInput):
    url_path = "/vision/v3.2/analyze"
    visualFeatures = ServiceParam("what visual feature types to return", url_param=True)
    details = ServiceParam("what visual feature types to return", url_param=True)
    language = ServiceParam("the language of the response (en if none given)", url_param=True)
    descriptionExclude = ServiceParam("Whether to exclude certain parameters from the description",
                                      url_param=True)

    def _query(self, vals):
        q = []
        for k in ("visualFeatures", "details", "descriptionExclude"):
            if k in vals:
                v = vals[k]
                q.append((k, ",".join(v) if isinstance(v, (list, tuple)) else str(v)))
        if "language" in vals:
            q.append(("language", vals["language"]))
        return q


class OCR(_ImageInput):
    url_path = "/vision/v3.2/ocr"
    language = ServiceParam("The BCP-47 language code of the text to be detected in the image", url_param=True)
    detectOrientation = ServiceParam("Whether detect the text orientation in the image", url_param=True)


class ReadImage(_ImageInput, HasAsyncReply):
    url_path = "/vision/v3.2/read/analyze"
    language = ServiceParam("IThe BCP-47 language code of the text in the document.", url_param=True)
    readingOrder = ServiceParam("Optional parameter to specify which reading order algorithm should be applied "
                                "when ordering the extract text elements", url_param=True)


class RecognizeText(ReadImage):
    """Deprecated alias kept by the reference; uses the Read API."""


class DescribeImage(_ImageInput):
    url_path = "/vision/v3.2/describe"
    maxCandidates = ServiceParam("Maximum candidate descriptions to be returned", url_param=True)
    language = ServiceParam("Language of image description", url_param=True)


class TagImage(_ImageInput):
    url_path = "/vision/v3.2/tag"
    language = ServiceParam("The desired language for output generation.", url_param=True)


class RecognizeDomainSpecificContent(_ImageInput):
    url_path = "/vision/v3.2/models/"
    model = ServiceParam("the domain specific model: celebrities, landmarks", required=True)

    def _base_url(self, vals):
        return self.getUrl().rstrip("/") + "/" + vals["model"] + "/analyze"


class GenerateThumbnails(_ImageInput):
    url_path = "/vision/v3.2/generateThumbnail"
    width = ServiceParam("the desired width of the image", required=True, url_param=True)
    height = ServiceParam("the desired height of the thumbnail", required=True, url_param=True)
    smartCropping = ServiceParam("whether to intelligently crop the image", url_param=True)

    def _should_skip(self, vals):
        return super()._should_skip(vals) or "width" not in vals or "height" not in vals

    def _parse(self, resp):
        return resp["entity"]["content"] if resp.get("entity") else None


# ---------------------------------------------------------------------- Face
class DetectFace(_ImageInput):
    url_path = "/face/v1.0/detect"
    returnFaceId = ServiceParam("Return faceIds of the detected faces or not", url_param=True)
    returnFaceLandmarks = ServiceParam("Return face landmarks of the detected faces or not", url_param=True)
    returnFaceAttributes = ServiceParam("Analyze and return the one or more specified face attributes",
                                        url_param=True)
    recognitionModel = ServiceParam("The recognition model", url_param=True)
    detectionModel = ServiceParam("The detection model", url_param=True)
    returnRecognitionModel = ServiceParam("whether to return the recognition model", url_param=True)

    def _query(self, vals):
        q = super()._query({k: v for k, v in vals.items() if k != "returnFaceAttributes"})
        if "returnFaceAttributes" in vals:
            v = vals["returnFaceAttributes"]
            q.append(("returnFaceAttributes", ",".join(v) if isinstance(v, (list, tuple)) else str(v)))
        return q


class FindSimilarFace(CognitiveServicesBase):
    url_path = "/face/v1.0/findsimilars"
    faceId = ServiceParam("faceId of the query face", required=True)
    faceListId = ServiceParam("An existing user-specified unique candidate face list")
    largeFaceListId = ServiceParam("An existing user-specified unique candidate large face list")
    faceIds = ServiceParam("An array of candidate faceIds")
    maxNumOfCandidatesReturned = ServiceParam("The number of top similar faces returned")
    mode = ServiceParam("Similar face searching mode: matchPerson or matchFace")


class GroupFaces(CognitiveServicesBase):
    url_path = "/face/v1.0/group"
    faceIds = ServiceParam("Array of candidate faceId created by Face - Detect", required=True)


class IdentifyFaces(CognitiveServicesBase):
    url_path = "/face/v1.0/identify"
    faceIds = ServiceParam("Array of query faces faceIds", required=True)
    personGroupId = ServiceParam("personGroupId of the target person group")
    largePersonGroupId = ServiceParam("largePersonGroupId of the target large person group")
    maxNumOfCandidatesReturned = ServiceParam("The range of maxNumOfCandidatesReturned is between 1 and 100")
    confidenceThreshold = ServiceParam("Customized identification confidence threshold, in the range [0, 1]")


class VerifyFaces(CognitiveServicesBase):
    url_path = "/face/v1.0/verify"
    faceId1 = ServiceParam("faceId of one face")
    faceId2 = ServiceParam("faceId of another face")
    faceId = ServiceParam("faceId of the face")
    personGroupId = ServiceParam("Using existing personGroupId and personId for fast loading")
    largePersonGroupId = ServiceParam("Using existing largePersonGroupId and personId")
    personId = ServiceParam("Specify a certain person in a person group")


__all__ = ["AnalyzeImage", "OCR", "ReadImage", "RecognizeText", "DescribeImage", "TagImage",
           "RecognizeDomainSpecificContent", "GenerateThumbnails", "DetectFace", "FindSimilarFace", "GroupFaces",
           "IdentifyFaces", "VerifyFaces"]
